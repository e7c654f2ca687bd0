#!/bin/bash
# GPU: the deflate parity tests, then the C2 step at 512..4096 streams with one- and two-wave parses
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/pw
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_deflate.py -k "two_wave or small_goldens or c2_full" > gpurun_out/pw/test.log 2>&1 || { tail -30 gpurun_out/pw/test.log; exit 1; }
tail -1 gpurun_out/pw/test.log
for s in 512 1024 2048 4096; do for w in 1 2 4; do
  timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-shard-sweep --no-e2e --streams $s --option parse_waves=$w > gpurun_out/pw/b_${s}_$w.log 2>&1 || { tail -5 gpurun_out/pw/b_${s}_$w.log; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['ms_per_step'], d['roofline']['phase_ms'], d['verify']['mismatches'])" gpurun_out/pw/b_${s}_$w.log "$s w=$w"
done; done
