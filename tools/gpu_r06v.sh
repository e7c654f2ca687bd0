#!/bin/bash
# round 6: the 768-bit sync window (20 KB of LDS per walk: eight walks per CU) vs 1024 (six)
set -o pipefail
O=gpurun_out/r06v; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_seg.py -x -q --timeout 300 --timeout-method thread > $O/test.log 2>&1 || { tail -30 $O/test.log; exit 1; }
tail -2 $O/test.log
TAG=r06v_narrow bash tools/dec_shards.sh --option seg_narrow=1 > $O/dec_shards_narrow.txt 2>&1 || exit 1
cat $O/dec_shards_narrow.txt
TAG=r06v bash tools/dec_shards.sh > $O/dec_shards.txt 2>&1 || exit 1
cat $O/dec_shards.txt
echo done
