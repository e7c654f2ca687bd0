#!/bin/bash
# Kernel-trace pass (rocprofv3 --kernel-trace --stats) of a short bench run.
# usage: tools/trace.sh OUTDIR [bench args...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=$1; shift
mkdir -p "$OUT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- python3 bench.py --no-cpu-baseline --no-shard-sweep --no-e2e --no-verify --steps 3 --warmup 1 "$@" > "$OUT/trace.log" 2>&1 || exit $?
python3 tools/summarize_profile.py "$OUT" "$OUT/summary.json"
