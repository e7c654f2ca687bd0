#!/bin/bash
# round 6: the whole GPU suite at this build, then the decode shards
set -o pipefail
O=gpurun_out/r06m; mkdir -p $O
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gputest.log 2>&1 || { tail -30 $O/gputest.log; exit 1; }
TAG=r06m bash tools/dec_shards.sh > $O/dec_shards.txt 2>&1 || exit 1
echo done
