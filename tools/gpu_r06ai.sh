#!/bin/bash
# round 6: the lazy parse's waves per stream at 512 and 1,024 streams (default two)
set -o pipefail
O=gpurun_out/r06ai; mkdir -p $O
X="--steps 20 --warmup 3 --no-cpu-baseline --no-e2e --no-shard-sweep"
for n in 512 1024; do
for pw in 1 2 1 2; do
  timeout -k 10 300 python bench.py $X --streams $n --option parse_waves=$pw > $O/c2_${n}_pw$pw.log 2>&1 || exit 1
  python3 -c "import json; d=json.loads(open('$O/c2_${n}_pw$pw.log').read().strip().splitlines()[-1]); print('$n pw$pw', d['ms_per_step'], d['roofline']['phase_ms']['parse'], d['verify']['mismatches'])"
done
done
echo done
