#!/bin/bash
# round 6: the lazy parse's waves per stream at 4,096 streams (default one) and at 2,048 (default two)
set -o pipefail
O=gpurun_out/r06ah; mkdir -p $O
X="--steps 10 --warmup 3 --no-cpu-baseline --no-e2e --no-shard-sweep"
for pw in 1 2 4; do
  timeout -k 10 300 python bench.py $X --option parse_waves=$pw > $O/c2_pw$pw.log 2>&1 || exit 1
  python3 -c "import json; d=json.loads(open('$O/c2_pw$pw.log').read().strip().splitlines()[-1]); print('4096 pw$pw', d['ms_per_step'], d['roofline']['phase_ms']['parse'], d['verify']['mismatches'])"
done
for pw in 1 2; do
  timeout -k 10 300 python bench.py $X --streams 2048 --option parse_waves=$pw > $O/c2_2048_pw$pw.log 2>&1 || exit 1
  python3 -c "import json; d=json.loads(open('$O/c2_2048_pw$pw.log').read().strip().splitlines()[-1]); print('2048 pw$pw', d['ms_per_step'], d['roofline']['phase_ms']['parse'], d['verify']['mismatches'])"
done
echo done
