#!/bin/bash
# round 6: the decode ring at 64 values per lane (12 KB per wave with the capped table) vs 32
set -o pipefail
O=gpurun_out/r06ag; mkdir -p $O
ZS_LIB=variants/ring64/libzsgpu.so timeout -k 10 600 python -u -m pytest tests/test_gpu_seg.py -x -q --timeout 200 --timeout-method thread > $O/test64.log 2>&1 || { tail -30 $O/test64.log; exit 1; }
tail -1 $O/test64.log
ZS_LIB=variants/ring64/libzsgpu.so TAG=r06ag_ring64 bash tools/dec_shards.sh > $O/dec_shards_ring64.txt 2>&1 || exit 1
cat $O/dec_shards_ring64.txt
TAG=r06ag bash tools/dec_shards.sh > $O/dec_shards.txt 2>&1 || exit 1
cat $O/dec_shards.txt
echo done
