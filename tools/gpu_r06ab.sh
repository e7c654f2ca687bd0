#!/bin/bash
# round 6: the decode ring rows padded by 16 B (bank conflicts), vs the committed build
set -o pipefail
O=gpurun_out/r06ab; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_seg.py tests/test_gpu_inflate.py -x -q --timeout 200 --timeout-method thread > $O/test.log 2>&1 || { tail -30 $O/test.log; exit 1; }
tail -2 $O/test.log
TAG=r06ab bash tools/dec_shards.sh > $O/dec_shards.txt 2>&1 || exit 1
cat $O/dec_shards.txt
echo done
