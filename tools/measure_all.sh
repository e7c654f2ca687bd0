#!/bin/bash
# The round's measurement set on one MI355X (run through gpurun): headline bench
# with shard sweep / e2e / CPU baseline, the other BASELINE configs, and the
# rocprofv3 kernel trace + PMC passes of the headline.  Logs under $1.
# usage: tools/measure_all.sh OUTDIR [benches|profiles|all]
set -u
OUT=$1
WHAT=${2:-all}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p "$OUT"
run() {  # name seconds command...
  local name=$1 secs=$2; shift 2
  echo "=== $name"
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  tail -n 1 "$OUT/$name.log" | cut -c1-300
  if [ $rc -ne 0 ]; then echo "=== $name failed ($rc)"; exit $rc; fi
}
if [ "$WHAT" != profiles ]; then
run c2_headline 400 python3 bench.py
run c3_inflate 200 python3 bench.py --mode inflate --no-shard-sweep --no-e2e
run c5_gunzip 200 python3 bench.py --mode inflate --format gzip --streams 8192 --replicas 1 --no-shard-sweep --no-e2e
run c5_d64 200 python3 bench.py --mode inflate --format deflate64-raw --streams 8192 --replicas 1 --no-shard-sweep --no-e2e
run c5_gzip_l6 200 python3 bench.py --format gzip --streams 1024 --no-shard-sweep --no-e2e
run c4_l9 300 python3 bench.py --streams 512 --stream-bytes 262144 --level 9 --no-shard-sweep --no-e2e
run c4_l1 300 python3 bench.py --streams 512 --stream-bytes 262144 --level 1 --no-shard-sweep --no-e2e
fi
if [ "$WHAT" != benches ]; then
run profile 600 tools/profile.sh "$OUT/prof"
run prof_inflate 600 tools/profile.sh "$OUT/prof_inflate" --mode inflate
run sq 600 tools/pmc_sq.sh "$OUT/sq"
fi
echo measure-done
