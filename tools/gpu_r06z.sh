#!/bin/bash
# round 6: zs_k_bucket's passes (wall clock per workgroup), 4,096 and 512 streams
set -o pipefail
O=gpurun_out/r06z; mkdir -p $O
ZS_LIB=variants/bk/libzsgpu.so timeout -k 10 300 python tools/dbg/bucket_prof.py 4096 > $O/bk_4096.log 2>&1 || { tail -5 $O/bk_4096.log; exit 1; }
cat $O/bk_4096.log | grep us
ZS_LIB=variants/bk2/libzsgpu.so timeout -k 10 300 python tools/dbg/bucket_prof.py 4096 > $O/bk_512.log 2>&1 || exit 1
cat $O/bk_512.log | grep us
echo done
