#!/bin/bash
# round 6, first GPU call: the new capacity tests, the demand parse's phase profile, a baseline C2 bench
set -o pipefail
mkdir -p gpurun_out/r06a
timeout -k 10 300 python -u -m pytest tests/test_gpu_boundary.py -x -q --timeout 120 --timeout-method thread -k "exact_unaligned or unaligned or explicit_cap" > gpurun_out/r06a/test_caps.log 2>&1 || exit 1
for n in 4096 512; do
  ZS_LIB=variants/pp/libzsgpu.so timeout -k 10 120 python3 tools/parse_prof.py $n 0 1 > gpurun_out/r06a/pp_dw_$n.log 2>&1 || exit 1
  ZS_LIB=variants/pp/libzsgpu.so timeout -k 10 120 python3 tools/parse_prof.py $n 0 0 > gpurun_out/r06a/pp_def_$n.log 2>&1 || exit 1
done
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/r06a/bench_c2.log 2>&1 || exit 1
echo done
