#!/bin/bash
# round 6: the walk's wave-coherent stretch (every running lane between its windows: bookkeeping-free
# decode) vs without it (ZS_SEG_EXP=32)
set -o pipefail
O=gpurun_out/r06u; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_seg.py tests/test_gpu_inflate.py tests/test_gpu_split.py -x -q --timeout 300 --timeout-method thread > $O/test.log 2>&1 || { tail -30 $O/test.log; exit 1; }
tail -2 $O/test.log
TAG=r06u bash tools/dec_shards.sh > $O/dec_shards.txt 2>&1 || exit 1
cat $O/dec_shards.txt
echo done
