# segmented-decode diagnostics (gpurun): decode clocks of the instrumented build, then the GPU checks + shard benches
set -u
ZS_LIB=variants/segexp/libzsgpu.so timeout -k 10 200 python3 tools/dbg/seg_clock.py 512 262144 > gpurun_out/seg_clock.log 2>&1; cat gpurun_out/seg_clock.log
tools/gpu_seg_check.sh gpurun_out/r04f
