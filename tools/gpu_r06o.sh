#!/bin/bash
# round 6: the one-wave parse's staging window (occupancy): WIN 16 / 24 vs 32 on C2
set -o pipefail
O=gpurun_out/r06o; mkdir -p $O
X="--steps 10 --warmup 3 --no-cpu-baseline --no-e2e --no-shard-sweep"
for v in default pw16 pw24 default; do
  if [ $v = default ]; then L=""; else L=variants/$v/libzsgpu.so; fi
  ZS_LIB=$L timeout -k 10 300 python bench.py $X > $O/c2_$v.log 2>&1 || exit 1
  python3 -c "import json; d=json.loads(open('$O/c2_$v.log').read().strip().splitlines()[-1]); print('$v', d['ms_per_step'], d['roofline']['phase_ms']['parse'], d['verify']['mismatches'])"
done
echo done
