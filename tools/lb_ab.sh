#!/bin/bash
# C5-i gunzip / C5-ii deflate64 bench per (library, lane_block): tools/lb_ab.sh "LIB..." "LB..."
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/lbab
B="--no-cpu-baseline --no-shard-sweep --no-e2e --steps 5 --warmup 2 --mode inflate --streams 8192 --replicas 1"
for lib in $1; do
  for lb in $2; do
    for fmt in gzip deflate64-raw; do
      f=gpurun_out/lbab/$(echo "$lib" | tr '/' '_')_${lb}_$fmt.log
      ZS_LIB=$lib timeout -k 10 200 python3 bench.py $B --format $fmt --option lane_block=$lb > $f 2>&1 || { echo "$lib $lb $fmt failed"; tail -3 $f; exit 1; }
      echo "$lib lb=$lb $fmt $(tail -n 1 $f | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["ms_per_step"], d["verify"]["mismatches"], d["roofline"]["phase_ms"].get("inflate_lane"))')"
    done
  done
done
