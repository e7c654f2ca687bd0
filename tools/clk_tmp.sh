cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/clk3
tools/quick_deflate.sh || exit 1
for v in clk clk2; do
ZS_LIB=$PWD/zlib-streams-ts_amd/libzsgpu_$v.so timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-shard-sweep --no-e2e --no-verify --steps 2 --warmup 1 > gpurun_out/clk3/$v.log 2>&1 || exit 1
python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], d['roofline']['phase_ms']['bucket'])" gpurun_out/clk3/$v.log
done
