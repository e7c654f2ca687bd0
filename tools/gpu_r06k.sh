#!/bin/bash
# round 6: multi-piece resolve rounds -- seg/inflate/boundary suites, decode shards (split auto / on)
set -o pipefail
O=gpurun_out/r06k; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_seg.py tests/test_gpu_inflate.py tests/test_gpu_split.py -x -q --timeout 300 --timeout-method thread > $O/test.log 2>&1 || { tail -30 $O/test.log; exit 1; }
timeout -k 10 900 python -u -m pytest tests/test_gpu_boundary.py -x -q --timeout 600 --timeout-method thread -k "shard or large_member or c5 or gunzip or c3" > $O/test_boundary.log 2>&1 || { tail -30 $O/test_boundary.log; exit 1; }
TAG=r06k bash tools/dec_shards.sh > $O/dec_shards.txt 2>&1 || exit 1
TAG=r06k_s1 bash tools/dec_shards.sh --option seg_split=1 > $O/dec_shards_split1.txt 2>&1 || exit 1
echo done
