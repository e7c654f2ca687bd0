#!/bin/bash
# A/B of libzsgpu.so builds on the 4,096 x 256 KiB L6 decode (timing only): tools/ab_c4d.sh LIB...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/abd
for lib in "$@"; do
  tag=$(echo "$lib" | tr '/' '_')
  ZS_LIB=$lib timeout -k 10 300 python3 bench.py --mode inflate --stream-bytes 262144 --streams 4096 --replicas 1 --corpus text --no-cpu-baseline --no-shard-sweep --no-e2e --steps 3 --warmup 1 $ABD_EXTRA > gpurun_out/abd/$tag.log 2>&1 || { echo "$lib failed"; tail -3 gpurun_out/abd/$tag.log; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['ms_per_step'], d['verify']['mismatches'])" gpurun_out/abd/$tag.log "$lib"
done
