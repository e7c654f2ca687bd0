#!/bin/bash
# round 6: the walk's checkpoint spacing 256 bits (25 KB of LDS: six walks per CU) vs 128
set -o pipefail
O=gpurun_out/r06n; mkdir -p $O
ZS_LIB=variants/ckb256/libzsgpu.so timeout -k 10 600 python -u -m pytest tests/test_gpu_seg.py -x -q --timeout 300 --timeout-method thread > $O/test.log 2>&1 || { tail -30 $O/test.log; exit 1; }
ZS_LIB=variants/ckb256/libzsgpu.so TAG=r06n_ckb256 bash tools/dec_shards.sh > $O/dec_shards_ckb256.txt 2>&1 || exit 1
TAG=r06n bash tools/dec_shards.sh > $O/dec_shards.txt 2>&1 || exit 1
echo done
