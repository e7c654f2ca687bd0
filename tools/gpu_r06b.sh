#!/bin/bash
# round 6: the deflate suite and the seg option tests after pruning, then the C2 bench
set -o pipefail
mkdir -p gpurun_out/r06b
timeout -k 10 900 python -u -m pytest tests/test_gpu_deflate.py tests/test_gpu_seg.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r06b/test.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/r06b/bench_c2.log 2>&1 || exit 1
echo done
