#!/bin/bash
# GPU check of an inflate-kernel change: parity tests, C3 / C5-i rates (tools/quick_inflate.sh),
# the C5-ii deflate64 rate and the single largest deflate64 fixture
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
tools/quick_inflate.sh || exit 1
timeout -k 10 200 python3 bench.py --mode inflate --format deflate64-raw --streams 8192 --replicas 1 --no-shard-sweep --no-e2e --no-cpu-baseline > gpurun_out/quicki/c5d64.log 2>&1 || { tail -5 gpurun_out/quicki/c5d64.log; exit 1; }
python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('C5-ii', d['value'], d['roofline']['phase_ms'], d['verify'])" gpurun_out/quicki/c5d64.log
timeout -k 10 120 python3 tools/d64_single.py
