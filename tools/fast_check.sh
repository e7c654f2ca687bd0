#!/bin/bash
# GPU check of the L1-3 parser: its parity tests, then the C4 L1 bench (512 x 256 KiB) for both kernels
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/fast
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_deflate.py -k "group_fast or small_goldens or random_inputs or block_boundaries" > gpurun_out/fast/test.log 2>&1 || { tail -30 gpurun_out/fast/test.log; exit 1; }
tail -1 gpurun_out/fast/test.log
for g in 1 0; do
  timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-shard-sweep --no-e2e --streams 512 --stream-bytes 262144 --level 1 --option fast_group=$g "$@" > gpurun_out/fast/b_$g.log 2>&1 || { tail -5 gpurun_out/fast/b_$g.log; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], d['roofline']['phase_ms'], d['verify'])" gpurun_out/fast/b_$g.log "fast_group=$g"
done
