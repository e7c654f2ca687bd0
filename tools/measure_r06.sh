#!/bin/bash
# Round-6 measurement set on one MI355X (run through gpurun): the GPU suite, every
# BASELINE config's bench line (inflate configs with their per-rank shard sweeps),
# rocprofv3 kernel trace + FETCH/WRITE passes and SQ passes.  Logs under $1; copy
# the summaries into profiles/r06/ with tools/collect_r06.sh.
# usage: tools/measure_r06.sh OUTDIR [tests|benches|ibenches|dbenches|profiles[12]|sq[12]|rehearsal|all]...
set -u
OUT=$1; shift
WHAT=${*:-all}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p "$OUT"
want() { for w in $WHAT; do [ "$w" = "$1" ] || [ "$w" = all ] && return 0; done; return 1; }
run() {  # name seconds command...
  local name=$1 secs=$2; shift 2
  echo "=== $name"
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  tail -n 1 "$OUT/$name.log" | cut -c1-400
  if [ $rc -ne 0 ]; then echo "=== $name failed ($rc)"; exit $rc; fi
}
C3="--mode inflate"
C4D="--mode inflate --stream-bytes 262144 --streams 4096 --replicas 1 --corpus text"
C5I="--mode inflate --format gzip --streams 8192 --replicas 1"
C5D="--mode inflate --format deflate64-raw --streams 8192 --replicas 1"
C5G="--format gzip --streams 8192"
C4L9="--streams 512 --stream-bytes 262144 --level 9"
C4L1="--streams 512 --stream-bytes 262144 --level 1"
if want tests; then
run gputest 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
fi
if want ibenches || want benches; then
run c4_decode 400 python3 bench.py $C4D --no-e2e
run c5_gunzip 300 python3 bench.py $C5I --no-e2e
run c5_d64 300 python3 bench.py $C5D --no-e2e
run c3_inflate 300 python3 bench.py $C3 --no-shard-sweep
fi
if want dbenches || want benches; then
run c2_headline 400 python3 bench.py
run c5_gzip_l6 200 python3 bench.py $C5G --no-shard-sweep --no-e2e
run c4_l9 300 python3 bench.py $C4L9 --no-shard-sweep --no-e2e
run c4_l1 300 python3 bench.py $C4L1 --no-shard-sweep --no-e2e
fi
if want profiles || want profiles1; then
run prof_c2 300 tools/profile.sh "$OUT/prof_c2"
run prof_c3 300 tools/profile.sh "$OUT/prof_c3" $C3
run prof_c4_decode 300 tools/profile.sh "$OUT/prof_c4_decode" $C4D
run prof_c5_gunzip 300 tools/profile.sh "$OUT/prof_c5_gunzip" $C5I
fi
if want profiles || want profiles2; then
run prof_c5_d64 300 tools/profile.sh "$OUT/prof_c5_d64" $C5D
run prof_c5_gzip_l6 300 tools/profile.sh "$OUT/prof_c5_gzip_l6" $C5G
run prof_c4_l9 300 tools/profile.sh "$OUT/prof_c4_l9" $C4L9
run prof_c4_l1 300 tools/profile.sh "$OUT/prof_c4_l1" $C4L1
fi
if want sq || want sq1; then
run sq_c2 500 tools/pmc_sq.sh "$OUT/sq_c2"
run sq_c3 500 tools/pmc_sq.sh "$OUT/sq_c3" $C3
run sq_c4_decode 500 tools/pmc_sq.sh "$OUT/sq_c4_decode" $C4D
run sq_c5_gunzip 500 tools/pmc_sq.sh "$OUT/sq_c5_gunzip" $C5I
fi
if want sq || want sq2; then
run sq_c5_d64 500 tools/pmc_sq.sh "$OUT/sq_c5_d64" $C5D
run sq_c5_gzip_l6 500 tools/pmc_sq.sh "$OUT/sq_c5_gzip_l6" $C5G
run sq_c4_l9 500 tools/pmc_sq.sh "$OUT/sq_c4_l9" $C4L9
run sq_c4_l1 500 tools/pmc_sq.sh "$OUT/sq_c4_l1" $C4L1
fi
if want rehearsal; then
run smoke 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
ZS_BENCH_BACKEND=gloo run bench_2ranks_gloo_1gpu 400 python3 bench.py --gpus 2 --steps 5 --warmup 2 --no-cpu-baseline
ZS_BENCH_BACKEND=gloo run inflate_2ranks_gloo_1gpu 400 python3 bench.py --gpus 2 --mode inflate --steps 5 --warmup 2 --no-cpu-baseline
fi
echo measure-done
