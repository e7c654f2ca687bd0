#!/bin/bash
# GPU: the chunked-pipeline parity test, then the C2 step at several batch sizes x chunk counts
# usage: tools/chunk_sweep.sh "<chunk counts>" "<stream counts>" [bench args...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/chunks
KS=${1:-"1 2 4 8"}; NS=${2:-"512 4096"}; shift 2
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_deflate.py -k "chunked or small_goldens or c2_full" > gpurun_out/chunks/test.log 2>&1 || { tail -30 gpurun_out/chunks/test.log; exit 1; }
tail -1 gpurun_out/chunks/test.log
for s in $NS; do for k in $KS; do
  timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-shard-sweep --no-e2e --streams $s --option chunks=$k "$@" > gpurun_out/chunks/b_${s}_$k.log 2>&1 || { tail -5 gpurun_out/chunks/b_${s}_$k.log; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['ms_per_step'], d['roofline']['phase_ms'], d['verify']['mismatches'])" gpurun_out/chunks/b_${s}_$k.log "$s k=$k"
done; done
