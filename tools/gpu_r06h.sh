#!/bin/bash
# round 6: two-wave walks (128-lane spans) -- seg/inflate suites, decode shards
set -o pipefail
O=gpurun_out/r06h; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_seg.py tests/test_gpu_inflate.py tests/test_gpu_split.py -x -q --timeout 300 --timeout-method thread > $O/test.log 2>&1 || { tail -30 $O/test.log; exit 1; }
TAG=r06h bash tools/dec_shards.sh > $O/dec_shards.txt 2>&1 || exit 1
TAG=r06h_w1 bash tools/dec_shards.sh --option seg_waves=1 > $O/dec_shards_w1.txt 2>&1 || exit 1
echo done
