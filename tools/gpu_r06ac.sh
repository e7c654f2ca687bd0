#!/bin/bash
# round 6: the segmented decode's LDS ring at 16 values per lane (7.8 KB per wave: 20 waves per CU instead of 16)
set -o pipefail
O=gpurun_out/r06ac; mkdir -p $O
ZS_LIB=variants/ring16/libzsgpu.so timeout -k 10 600 python -u -m pytest tests/test_gpu_seg.py tests/test_gpu_inflate.py -x -q --timeout 200 --timeout-method thread > $O/test16.log 2>&1 || { tail -30 $O/test16.log; exit 1; }
tail -1 $O/test16.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_seg.py -x -q --timeout 200 --timeout-method thread > $O/test.log 2>&1 || { tail -30 $O/test.log; exit 1; }
tail -1 $O/test.log
ZS_LIB=variants/ring16/libzsgpu.so TAG=r06ac_ring16 bash tools/dec_shards.sh > $O/dec_shards_ring16.txt 2>&1 || exit 1
cat $O/dec_shards_ring16.txt
TAG=r06ac bash tools/dec_shards.sh > $O/dec_shards.txt 2>&1 || exit 1
cat $O/dec_shards.txt
echo done
