#!/bin/bash
# round 6: the walk without tail bitmaps (each tail start tested against the next lane's own starts, waiting for
# its word; 16 KB of LDS: eight walks per CU)
set -o pipefail
O=gpurun_out/r06w; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_seg.py -x -v --timeout 120 --timeout-method thread 2>&1 | tee $O/test_seg.log | grep -E "PASS|FAIL|ERROR|passed|failed" || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_inflate.py tests/test_gpu_split.py -x -q --timeout 200 --timeout-method thread > $O/test.log 2>&1 || { tail -30 $O/test.log; exit 1; }
tail -2 $O/test.log
TAG=r06w bash tools/dec_shards.sh > $O/dec_shards.txt 2>&1 || exit 1
cat $O/dec_shards.txt
echo done
