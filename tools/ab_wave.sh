#!/bin/bash
# A/B of libzsgpu.so builds on the wave-kernel benches (timing only): tools/ab_wave.sh LIB...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/abw
for lib in "$@"; do
  tag=$(echo "$lib" | tr '/' '_')
  ZS_LIB=$lib timeout -k 10 200 python3 bench.py --mode inflate --format deflate64-raw --streams 8192 --replicas 1 --no-shard-sweep --no-e2e --no-cpu-baseline --no-verify --steps 3 --warmup 1 > gpurun_out/abw/d64_$tag.log 2>&1 || { echo "$lib failed"; tail -3 gpurun_out/abw/d64_$tag.log; exit 1; }
  ZS_LIB=$lib timeout -k 10 200 python3 bench.py --mode inflate --stream-bytes 262144 --streams 4096 --replicas 1 --corpus text --no-cpu-baseline --no-shard-sweep --no-e2e --no-verify --steps 3 --warmup 1 > gpurun_out/abw/l256_$tag.log 2>&1 || { echo "$lib failed"; tail -3 gpurun_out/abw/l256_$tag.log; exit 1; }
  for t in d64 l256; do
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], sys.argv[3], d['ms_per_step'], d['roofline']['phase_ms'])" gpurun_out/abw/${t}_$tag.log "$lib" $t
  done
done
