#!/bin/bash
# round 6: the segmented decode's far copy rounds with their eight loads issued together (and provably near
# values read from the ring) vs a load-and-wait per value
set -o pipefail
O=gpurun_out/r06ao; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_seg.py tests/test_gpu_inflate.py tests/test_gpu_boundary.py -x -q --timeout 300 --timeout-method thread > $O/test.log 2>&1 || { tail -30 $O/test.log; exit 1; }
tail -1 $O/test.log
TAG=r06ao bash tools/dec_shards.sh > $O/dec_shards.txt 2>&1 || exit 1
cat $O/dec_shards.txt
ZS_LIB=variants/get0/libzsgpu.so TAG=r06ao_get0 bash tools/dec_shards.sh > $O/dec_shards_get0.txt 2>&1 || exit 1
cat $O/dec_shards_get0.txt
echo done
