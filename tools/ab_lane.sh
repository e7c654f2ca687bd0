#!/bin/bash
# A/B of libzsgpu.so builds on the lane-inflate benches C3 and C5-i (timing only): tools/ab_lane.sh LIB...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/abl
for lib in "$@"; do
  tag=$(echo "$lib" | tr '/' '_')
  for cfg in "c3:--mode inflate" "c5i:--mode inflate --format gzip --streams 8192 --replicas 1" "c5d:--mode inflate --format deflate64-raw --streams 8192 --replicas 1"; do
    name=${cfg%%:*}; args=${cfg#*:}
    ZS_LIB=$lib timeout -k 10 200 python3 bench.py $args --no-shard-sweep --no-e2e --no-cpu-baseline --no-verify --steps 5 --warmup 2 > gpurun_out/abl/${name}_$tag.log 2>&1 || { echo "$lib $name failed"; tail -3 gpurun_out/abl/${name}_$tag.log; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], sys.argv[3], d['ms_per_step'])" gpurun_out/abl/${name}_$tag.log "$lib" $name
  done
done
