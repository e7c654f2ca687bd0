#!/bin/bash
# GPU A/B of the demand-driven sweep (option demand): the deflate parity tests,
# then the headline batch and the 512-stream shard with demand on and off (phase
# times, golden verify) -- usage: tools/ab_demand.sh [bench args...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab_demand
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_deflate.py > gpurun_out/ab_demand/test.log 2>&1
rc=$?
tail -3 gpurun_out/ab_demand/test.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for s in 4096 512; do
  for d in 1 0; do
    timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-shard-sweep --no-e2e --streams $s --option demand=$d "$@" > gpurun_out/ab_demand/b_${s}_$d.log 2>&1 || { tail -5 gpurun_out/ab_demand/b_${s}_$d.log; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], 'demand', sys.argv[3], d['ms_per_step'], d['roofline']['phase_ms'], d['verify'])" gpurun_out/ab_demand/b_${s}_$d.log $s $d
  done
done
