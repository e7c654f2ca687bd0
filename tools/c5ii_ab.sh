#!/bin/bash
# C5-ii phase A/B: the C5-ii members (the T-corpus raw-L6 streams decoded as deflate64) with all of the
# reference's deflate64 fixtures, without them, and with one fixture at a time (which one lengthens the
# segmented decode's chain)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/c5ii_ab; mkdir -p $O
pr() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['ms_per_step'], {k: v for k, v in d['roofline']['phase_ms'].items() if v > 0.05})" "$@"; }
X="--mode inflate --format deflate64-raw --streams 8192 --replicas 1 --no-cpu-baseline --no-e2e --no-shard-sweep"
V=("base:" "nofix:--no-fixtures")
for f in ${C5_FIX:-100k_lines 10k_lines payload_63k payload_64k payload_65k rand_block repeat_63k repeat_64k repeat_65k zeros_100k}; do
  V+=("$f:--fixtures $f")
done
for v in "${V[@]}"; do
  n=${v%%:*}; a=${v#*:}
  timeout -k 10 300 python3 bench.py $X $a > $O/$n.log 2>&1 || { tail -3 $O/$n.log; exit 1; }
  pr $O/$n.log "$n"
done
