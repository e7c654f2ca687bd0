#!/bin/bash
# lane_block sweep of the narrow lane-inflate configs (C5-i gunzip, C5-ii deflate64): one bench line each.
# usage: tools/lb_sweep.sh OUTDIR
set -u
OUT=$1
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p "$OUT"
B="--no-cpu-baseline --no-shard-sweep --no-e2e --steps 5 --warmup 2 --mode inflate --streams 8192 --replicas 1"
for lb in 1 2 4; do
  for fmt in gzip deflate64-raw; do
    timeout -k 10 200 python3 bench.py $B --format $fmt --option lane_block=$lb > "$OUT/lb${lb}_$fmt.log" 2>&1 || exit $?
    echo "lb=$lb $fmt $(tail -n 1 "$OUT/lb${lb}_$fmt.log" | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["ms_per_step"], d["roofline"].get("phase_ms"))')"
  done
done
