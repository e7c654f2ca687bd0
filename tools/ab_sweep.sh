#!/bin/bash
# A/B of libzsgpu.so builds on the C2 bench (timing only): tools/ab_sweep.sh LIB...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab
for lib in "$@"; do
  tag=$(echo "$lib" | tr '/' '_')
  ZS_LIB=$lib timeout -k 10 120 python3 bench.py --no-cpu-baseline --no-shard-sweep --no-e2e --no-verify --steps 10 --warmup 3 > gpurun_out/ab/$tag.log 2>&1 || { echo "$lib failed"; tail -3 gpurun_out/ab/$tag.log; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['ms_per_step'], d['roofline']['phase_ms'])" gpurun_out/ab/$tag.log "$lib"
done
