#!/bin/bash
# Round-end evidence on one MI355X: the whole -m gpu suite, smoke(), then every BASELINE config's bench line.
# usage: tools/final_check.sh OUTDIR
set -u
OUT=$1
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p "$OUT"
echo "=== gpu tests $(date +%T)"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > "$OUT/gputest.log" 2>&1 || { tail -30 "$OUT/gputest.log"; exit 1; }
tail -1 "$OUT/gputest.log"
echo "=== smoke $(date +%T)"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { tail -20 "$OUT/smoke.log"; exit 1; }
tools/measure_all.sh "$OUT/bench" benches
