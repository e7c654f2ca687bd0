#!/bin/bash
# GPU A/B of the deflate chunk pipeline (option pipeline): the deflate parity tests, then the
# headline batch with 1 (off), 4 (default), 8 chunks -- usage: tools/ab_pipeline.sh [bench args...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/ab_pipe; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_deflate.py > $O/test.log 2>&1
rc=$?; tail -2 $O/test.log; [ $rc -eq 0 ] || exit $rc
for k in 1 4 8 2; do
  timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-shard-sweep --no-e2e --option pipeline=$k "$@" > $O/b_$k.log 2>&1 || { tail -5 $O/b_$k.log; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('pipeline', sys.argv[2], d['ms_per_step'], d['value'], d['roofline']['phase_ms'], d['verify']['mismatches'])" $O/b_$k.log $k
done
