set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_deflate.py > gpurun_out/ab/test.log 2>&1
tail -2 gpurun_out/ab/test.log
for w in 0 16 32; do
 for s in 4096 512; do
  timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-shard-sweep --no-e2e --streams $s --option parse_win=$w > gpurun_out/ab/b_${w}_${s}.log 2>&1
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], sys.argv[3], d['ms_per_step'], d['roofline']['phase_ms']['parse'], d['verify'])" gpurun_out/ab/b_${w}_${s}.log $w $s
 done
done
