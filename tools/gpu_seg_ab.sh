#!/bin/bash
# A/B of segmented-decode options on one config (gpurun): prints the step and phases per option set.
# usage: tools/gpu_seg_ab.sh OUTDIR "bench args" "opt1 opt2" "opt3" ...   (each quoted group: --option values)
set -u
OUT=$1; ARGS=$2; shift 2
mkdir -p "$OUT"
i=0
for g in "" "$@"; do
  o=""
  for kv in $g; do o="$o --option $kv"; done
  timeout -k 10 200 python3 bench.py $ARGS --no-shard-sweep --no-e2e --no-cpu-baseline $o > "$OUT/ab_$i.log" 2>&1 || { tail -3 "$OUT/ab_$i.log"; exit 1; }
  python3 - "$OUT/ab_$i.log" "$g" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().split("\n")[-1])
print(repr(sys.argv[2]), d["ms_per_step"], {k: v for k, v in d["roofline"]["phase_ms"].items() if v > 0.05})
PY
  i=$((i+1))
done
