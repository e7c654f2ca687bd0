set -e
cd "${GRAFT_REPO_ROOT}"
tools/ab_sweep.sh zlib-streams-ts_amd/libzsgpu.so variants/bksplit/libzsgpu.so zlib-streams-ts_amd/libzsgpu.so variants/bksplit/libzsgpu.so
ZS_LIB=variants/bksplit/libzsgpu.so timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-e2e > gpurun_out/ab/bksplit_verify.log 2>&1
tail -1 gpurun_out/ab/bksplit_verify.log | cut -c1-100
python3 -c "import json; d=json.loads(open('gpurun_out/ab/bksplit_verify.log').read().strip().splitlines()[-1]); print(d['verify'], d['shard_sweep_ms'], d['roofline']['phase_ms'])"
