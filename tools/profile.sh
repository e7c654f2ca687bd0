#!/bin/bash
# rocprofv3 passes for the bench workload (run on the GPU box via gpurun):
#   1) kernel trace + stats, 2) FETCH_SIZE, 3) WRITE_SIZE (separate PMC passes,
#   MI355X_MICROARCH.md "rocprofv3 PMC slots" / "HBM").
# usage: tools/profile.sh OUTDIR [bench args...]
set -u
OUT=$1; shift
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p "$OUT"
ARGS="--no-cpu-baseline --no-shard-sweep --no-e2e --no-verify --steps 10 --warmup 1 $*"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- python3 bench.py $ARGS > "$OUT/trace.log" 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o run -- python3 bench.py $ARGS > "$OUT/fetch.log" 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o run -- python3 bench.py $ARGS > "$OUT/write.log" 2>&1 || exit $?
python3 tools/summarize_profile.py "$OUT" "$OUT/summary.json"
echo profile-done
