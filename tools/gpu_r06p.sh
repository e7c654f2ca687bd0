#!/bin/bash
# round 6: the walk's fast stretch between the two sync windows vs without it (ZS_SEG_EXP=32)
set -o pipefail
O=gpurun_out/r06p; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_seg.py tests/test_gpu_inflate.py -x -q --timeout 300 --timeout-method thread > $O/test.log 2>&1 || { tail -30 $O/test.log; exit 1; }
tail -2 $O/test.log
TAG=r06p_fast bash tools/dec_shards.sh > $O/dec_shards_fast.txt 2>&1 || exit 1
cat $O/dec_shards_fast.txt
ZS_LIB=variants/nofast/libzsgpu.so TAG=r06p_nofast bash tools/dec_shards.sh > $O/dec_shards_nofast.txt 2>&1 || exit 1
cat $O/dec_shards_nofast.txt
echo done
