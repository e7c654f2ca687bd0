#!/bin/bash
# round 6: own-start chunks in the windowed sweep -- deflate suite, C4-L9 / C4-L1 shards, C2
set -o pipefail
O=gpurun_out/r06g; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_deflate.py -x -q --timeout 300 --timeout-method thread > $O/test.log 2>&1 || { tail -30 $O/test.log; exit 1; }
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-e2e --no-shard-sweep --stream-bytes 262144 --streams 512 --level 9 > $O/bench_c4l9.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-e2e --no-shard-sweep > $O/bench_c2.log 2>&1 || exit 1
echo done
