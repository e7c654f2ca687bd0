"""Cycle profile of zs_k_fast_mr's phases (a -DZS_FM_PROF build; prints from the kernel).  Runs 512 x 256 KiB
T-corpus streams (C4-L1's shard) so the CU sharing is the bench's; streams 0..3 print.

  make -C zlib-streams-ts_amd/csrc BUILD=build_prof OUT=../../variants/fmprof/libzsgpu.so \
       HIPFLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -DZS_FM_PROF"
  ZS_LIB=variants/fmprof/libzsgpu.so python3 tools/dbg/fm_prof.py 1
"""
import os
import sys
sys.path.insert(0, "zlib-streams-ts_amd")
import zsamd

lvl = int(sys.argv[1]) if len(sys.argv) > 1 else 1
eng = zsamd.Engine(0)
eng.set_option("fast_mr", 1)
buf = bytes(zsamd.corpus("text", 0, 512, 262144))
ins = [buf[i * 262144:(i + 1) * 262144] for i in range(512)]
eng.compress_batch_raw(ins, "deflate-raw", lvl)
