#!/bin/bash
# round 6: global / LDS typed pointers in the decoders (no flat loads of selected pointers, no scratch
# tables in zs_k_seg_decode, the walk's volatile LDS accesses as ds ops)
set -o pipefail
O=gpurun_out/r06q; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_seg.py tests/test_gpu_inflate.py tests/test_gpu_split.py tests/test_gpu_boundary.py -x -q --timeout 300 --timeout-method thread > $O/test.log 2>&1 || { tail -30 $O/test.log; exit 1; }
tail -2 $O/test.log
TAG=r06q bash tools/dec_shards.sh > $O/dec_shards.txt 2>&1 || exit 1
cat $O/dec_shards.txt
timeout -k 10 300 python bench.py --mode inflate --no-shard-sweep --no-cpu-baseline --no-e2e > $O/c3.log 2>&1 || exit 1
python3 -c "import json; d=json.loads(open('$O/c3.log').read().strip().splitlines()[-1]); print('C3', d['ms_per_step'], d['value'])"
echo done
