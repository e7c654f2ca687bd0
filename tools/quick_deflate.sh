#!/bin/bash
# GPU check of a deflate-kernel change: the deflate parity tests, then the headline
# bench and the 512-stream shard (phase times) -- usage: tools/quick_deflate.sh [bench args...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/quick
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_deflate.py > gpurun_out/quick/test.log 2>&1 || { tail -30 gpurun_out/quick/test.log; exit 1; }
tail -1 gpurun_out/quick/test.log
for s in 4096 512; do
  timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-shard-sweep --no-e2e --streams $s "$@" > gpurun_out/quick/b_$s.log 2>&1 || { tail -5 gpurun_out/quick/b_$s.log; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['ms_per_step'], d['roofline']['phase_ms'], d['verify'])" gpurun_out/quick/b_$s.log $s
done
