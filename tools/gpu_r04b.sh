set -u
mkdir -p gpurun_out/r04b
T="timeout -k 10"
$T 600 python3 -u -m pytest tests/test_gpu_deflate.py -m gpu -x -v --timeout 300 --timeout-method thread -k "ballot or selftest or group_fast or sweep_match" > gpurun_out/r04b/lane_order.log 2>&1 || { tail -5 gpurun_out/r04b/lane_order.log; exit 1; }
tail -2 gpurun_out/r04b/lane_order.log
C4D="--mode inflate --stream-bytes 262144 --replicas 1 --corpus text --no-shard-sweep --no-e2e --no-cpu-baseline"
C5I="--mode inflate --format gzip --replicas 1 --no-shard-sweep --no-e2e --no-cpu-baseline"
for n in 512 2048; do $T 200 python3 bench.py $C4D --streams $n > gpurun_out/r04b/c4d_$n.log 2>&1 || exit 1; done
for n in 1024 4096 8192; do $T 200 python3 bench.py $C5I --streams $n > gpurun_out/r04b/c5i_$n.log 2>&1 || exit 1; done
for n in 1024 4096 8192; do $T 200 python3 bench.py $C5I --streams $n --option inflate_seg=0 > gpurun_out/r04b/c5i_noseg_$n.log 2>&1 || exit 1; done
for n in 512 2048; do $T 200 python3 bench.py $C4D --streams $n --option inflate_seg=0 > gpurun_out/r04b/c4d_noseg_$n.log 2>&1 || exit 1; done
echo done
