#!/bin/bash
# A/B of libzsgpu.so builds on one bench config (timing, then a verified run of each
# variant): BENCH_ARGS="--streams 512" tools/ab_libs.sh TAG LIB...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
tag=$1; shift
mkdir -p gpurun_out/ab
for rep in 1 2; do
  for lib in "$@"; do
    t=$(echo "$lib" | tr '/' '_')
    ZS_LIB=$lib timeout -k 10 120 python3 bench.py --no-cpu-baseline --no-shard-sweep --no-e2e --no-verify --steps 10 --warmup 3 $BENCH_ARGS > gpurun_out/ab/${tag}_$t.log 2>&1 || { echo "$lib failed"; tail -3 gpurun_out/ab/${tag}_$t.log; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['ms_per_step'], d['roofline']['phase_ms'])" gpurun_out/ab/${tag}_$t.log "$lib"
  done
done
for lib in "$@"; do
  t=$(echo "$lib" | tr '/' '_')
  ZS_LIB=$lib timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-shard-sweep --no-e2e $BENCH_ARGS > gpurun_out/ab/${tag}_${t}_verify.log 2>&1 || { echo "$lib verify failed"; tail -3 gpurun_out/ab/${tag}_${t}_verify.log; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], 'verify', d['verify'])" gpurun_out/ab/${tag}_${t}_verify.log "$lib"
done
