#!/bin/bash
# round 6: zs_k_bucket with 512-thread workgroups (seven scatter waves beside the claiming one) -- the deflate
# GPU tests, C2 (bucket 1.54 ms with 256 threads) and C4-L9
set -o pipefail
O=gpurun_out/r06aa; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_deflate.py -x -q --timeout 300 --timeout-method thread > $O/test.log 2>&1 || { tail -30 $O/test.log; exit 1; }
tail -2 $O/test.log
X="--steps 10 --warmup 3 --no-cpu-baseline --no-e2e"
timeout -k 10 300 python bench.py $X > $O/c2.log 2>&1 || exit 1
python3 -c "import json; d=json.loads(open('$O/c2.log').read().strip().splitlines()[-1]); print('c2', d['ms_per_step'], d['roofline']['phase_ms']['bucket'], d['verify']['mismatches'], d.get('shard_sweep_ms'))"
timeout -k 10 300 python bench.py --streams 512 --stream-bytes 262144 --level 9 $X --no-shard-sweep > $O/l9.log 2>&1 || exit 1
python3 -c "import json; d=json.loads(open('$O/l9.log').read().strip().splitlines()[-1]); print('l9', d['ms_per_step'], d['roofline']['phase_ms'].get('bucket'), d['verify']['mismatches'])"
echo done
