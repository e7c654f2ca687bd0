#!/bin/bash
# round 6: resolve marker batching only with the 32 KiB ring (vs per-value load and pick everywhere)
set -o pipefail
O=gpurun_out/r06at; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_seg.py tests/test_gpu_inflate.py tests/test_gpu_boundary.py -x -q --timeout 300 --timeout-method thread > $O/test.log 2>&1 || { tail -30 $O/test.log; exit 1; }
tail -1 $O/test.log
TAG=r06at bash tools/dec_shards.sh > $O/dec_shards.txt 2>&1 || exit 1
cat $O/dec_shards.txt
ZS_LIB=variants/x128/libzsgpu.so TAG=r06at_x128 bash tools/dec_shards.sh > $O/dec_shards_x128.txt 2>&1 || exit 1
cat $O/dec_shards_x128.txt
echo done
