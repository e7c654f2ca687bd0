#!/bin/bash
# A/B of libzsgpu.so builds on the C3 inflate bench (timing only): tools/ab_inflate.sh LIB...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/abi
for lib in "$@"; do
  tag=$(echo "$lib" | tr '/' '_')
  ZS_LIB=$lib timeout -k 10 200 python3 bench.py --mode inflate --no-cpu-baseline --no-verify --steps 5 --warmup 2 $ZS_AB_ARGS > gpurun_out/abi/$tag.log 2>&1 || { echo "$lib failed"; tail -3 gpurun_out/abi/$tag.log; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['ms_per_step'], d['roofline']['phase_ms'])" gpurun_out/abi/$tag.log "$lib"
done
