#!/bin/bash
# round 6: large deflate64 members through the segmented decode (finder entries) -- d64 tests + C5-ii bench + shard
set -o pipefail
O=gpurun_out/r06f; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_seg.py tests/test_gpu_split.py tests/test_gpu_inflate.py -x -q --timeout 300 --timeout-method thread -k "64 or d64 or fixture or split" > $O/test.log 2>&1 || { tail -30 $O/test.log; exit 1; }
timeout -k 10 300 python3 bench.py --mode inflate --format deflate64-raw --streams 8192 --replicas 1 --no-cpu-baseline --no-e2e --steps 10 --warmup 3 > $O/c5ii.log 2>&1 || { tail -5 $O/c5ii.log; exit 1; }
python3 -c "import json,sys; d=json.loads(open('$O/c5ii.log').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['shard_sweep_ms'], d.get('shard8_phase_ms'), d.get('verify'))"
echo done
