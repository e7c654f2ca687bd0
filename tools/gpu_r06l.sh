#!/bin/bash
# round 6: the resolve with a 32 KiB ring / 256 threads (four members per CU) vs the 64 KiB / 512 one
set -o pipefail
O=gpurun_out/r06l; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_seg.py tests/test_gpu_inflate.py tests/test_gpu_split.py -x -q --timeout 300 --timeout-method thread > $O/test.log 2>&1 || { tail -30 $O/test.log; exit 1; }
TAG=r06l bash tools/dec_shards.sh > $O/dec_shards.txt 2>&1 || exit 1
ZS_LIB=variants/res64k/libzsgpu.so TAG=r06l_64k bash tools/dec_shards.sh > $O/dec_shards_64k.txt 2>&1 || exit 1
ZS_LIB=variants/res32k512/libzsgpu.so TAG=r06l_32k512 bash tools/dec_shards.sh > $O/dec_shards_32k512.txt 2>&1 || exit 1
echo done
