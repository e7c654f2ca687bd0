#!/bin/bash
# Re-measure the configs whose path changed late in round 3 (C4 decode: large-member lanes; C5-ii: split
# decode): bench lines, rocprofv3 kernel trace + FETCH/WRITE, SQ counters.  usage: tools/measure_r03b.sh OUTDIR
set -u
OUT=$1
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p "$OUT"
run() {
  local name=$1 secs=$2; shift 2
  echo "=== $name"
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  tail -n 1 "$OUT/$name.log" | cut -c1-200
  if [ $rc -ne 0 ]; then echo "=== $name failed ($rc)"; exit $rc; fi
}
C4D="--mode inflate --stream-bytes 262144 --streams 4096 --replicas 1 --corpus text"
C5D="--mode inflate --format deflate64-raw --streams 8192 --replicas 1"
run c4_decode 300 python3 bench.py $C4D --no-shard-sweep --no-e2e
run c5_d64 200 python3 bench.py $C5D --no-shard-sweep --no-e2e
run prof_c4_decode 300 tools/profile.sh "$OUT/prof_c4_decode" $C4D
run prof_c5_d64 300 tools/profile.sh "$OUT/prof_c5_d64" $C5D
run sq_c4_decode 500 tools/pmc_sq.sh "$OUT/sq_c4_decode" $C4D
echo measure-done
