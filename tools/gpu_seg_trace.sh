set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r04d
C4D="--mode inflate --stream-bytes 262144 --replicas 1 --corpus text --no-shard-sweep --no-e2e --no-cpu-baseline --no-verify --steps 3 --warmup 1 --streams 512"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04d/trace -o run -- python3 bench.py $C4D > gpurun_out/r04d/trace.log 2>&1 || exit 1
cat gpurun_out/r04d/trace/run_kernel_stats.csv | cut -c1-200 | head -20
