#!/bin/bash
# round 6: the segmented decode's table in LDS capped at the entries blocks use (1,024; 8 KB per wave: 20 waves
# per CU instead of 16)
set -o pipefail
O=gpurun_out/r06af; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_seg.py tests/test_gpu_inflate.py tests/test_gpu_boundary.py tests/test_gpu_split.py -x -q --timeout 300 --timeout-method thread > $O/test.log 2>&1 || { tail -30 $O/test.log; exit 1; }
tail -1 $O/test.log
TAG=r06af bash tools/dec_shards.sh > $O/dec_shards.txt 2>&1 || exit 1
cat $O/dec_shards.txt
echo done
