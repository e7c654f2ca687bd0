set -u
export ZS_LIB=variants/segexp/libzsgpu.so
timeout -k 10 200 python3 tools/dbg/seg_clock.py 512 262144 && timeout -k 10 200 python3 tools/dbg/seg_clock.py 512 262144 seg_bits=8192
