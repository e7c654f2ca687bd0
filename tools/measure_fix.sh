#!/bin/bash
# SQ passes for the inflate lane kernel (C3), then the C4-L9 and C5 deflate64 bench lines
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$1
mkdir -p "$OUT"
timeout -k 10 500 tools/pmc_sq.sh "$OUT/sq_c3" --mode inflate > "$OUT/sq_c3.log" 2>&1 || { tail -5 "$OUT/sq_c3.log"; exit 1; }
timeout -k 10 200 python3 bench.py --streams 512 --stream-bytes 262144 --level 9 --no-shard-sweep --no-e2e > "$OUT/c4_l9.log" 2>&1 || exit 1
timeout -k 10 200 python3 bench.py --mode inflate --format deflate64-raw --streams 8192 --replicas 1 --no-shard-sweep --no-e2e > "$OUT/c5_d64.log" 2>&1 || exit 1
echo done
