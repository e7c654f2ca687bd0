#!/bin/bash
# GPU check of an inflate-kernel change: the inflate parity tests, then C3 and C5-i (gunzip) rates
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/quicki
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_inflate.py > gpurun_out/quicki/test.log 2>&1 || { tail -30 gpurun_out/quicki/test.log; exit 1; }
tail -1 gpurun_out/quicki/test.log
timeout -k 10 200 python3 bench.py --mode inflate --no-shard-sweep --no-e2e --no-cpu-baseline "$@" > gpurun_out/quicki/c3.log 2>&1 || { tail -5 gpurun_out/quicki/c3.log; exit 1; }
python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('C3', d['value'], d['roofline']['phase_ms'], d['verify'])" gpurun_out/quicki/c3.log
timeout -k 10 200 python3 bench.py --mode inflate --format gzip --streams 8192 --replicas 1 --no-shard-sweep --no-e2e --no-cpu-baseline "$@" > gpurun_out/quicki/c5.log 2>&1 || { tail -5 gpurun_out/quicki/c5.log; exit 1; }
python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('C5', d['value'], d['roofline']['phase_ms'], d['verify'])" gpurun_out/quicki/c5.log
