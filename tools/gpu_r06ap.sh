#!/bin/bash
# round 6: the resolve waits for this round's values before issuing the next round's loads (vs issue-then-wait-for-all)
set -o pipefail
O=gpurun_out/r06ap; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_seg.py tests/test_gpu_inflate.py tests/test_gpu_boundary.py -x -q --timeout 300 --timeout-method thread > $O/test.log 2>&1 || { tail -30 $O/test.log; exit 1; }
tail -1 $O/test.log
TAG=r06ap bash tools/dec_shards.sh > $O/dec_shards.txt 2>&1 || exit 1
cat $O/dec_shards.txt
ZS_LIB=variants/w64/libzsgpu.so TAG=r06ap_w64 bash tools/dec_shards.sh > $O/dec_shards_w64.txt 2>&1 || exit 1
cat $O/dec_shards_w64.txt
echo done
