#!/bin/bash
# round 6: the wave-parallel table builder (zs_inftab.h) -- self-check, inflate/seg suites, header clocks, decode shards
set -o pipefail
O=gpurun_out/r06d; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_inflate.py tests/test_gpu_seg.py tests/test_gpu_split.py -x -q --timeout 300 --timeout-method thread > $O/test.log 2>&1 || { tail -30 $O/test.log; exit 1; }
ZS_LIB=variants/seghdr/libzsgpu.so timeout -k 10 200 python3 tools/dbg/seg_hdr_clock.py 512 262144 > $O/hdr_512.log 2>&1 || exit 1
ZS_LIB=variants/seghdr/libzsgpu.so timeout -k 10 200 python3 tools/dbg/seg_hdr_clock.py 1024 65536 gzip > $O/hdr_c5i.log 2>&1 || exit 1
TAG=r06d bash tools/dec_shards.sh > $O/dec_shards.txt 2>&1 || exit 1
echo done
