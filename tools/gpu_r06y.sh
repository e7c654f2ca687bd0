#!/bin/bash
# round 6: the bucket kernel's pass 2 with 16 claims in flight per wait vs 8
set -o pipefail
O=gpurun_out/r06y; mkdir -p $O
X="--steps 10 --warmup 3 --no-cpu-baseline --no-e2e --no-shard-sweep"
for v in default bk16 default bk16; do
  if [ $v = default ]; then L=""; else L=variants/$v/libzsgpu.so; fi
  ZS_LIB=$L timeout -k 10 300 python bench.py $X > $O/c2_$v.log 2>&1 || exit 1
  python3 -c "import json; d=json.loads(open('$O/c2_$v.log').read().strip().splitlines()[-1]); print('$v', d['ms_per_step'], d['roofline']['phase_ms']['bucket'], d['verify']['mismatches'])"
done
ZS_LIB=variants/bk16/libzsgpu.so timeout -k 10 300 python bench.py --streams 512 --stream-bytes 262144 --level 9 $X > $O/l9_bk16.log 2>&1 || exit 1
python3 -c "import json; d=json.loads(open('$O/l9_bk16.log').read().strip().splitlines()[-1]); print('l9 bk16', d['ms_per_step'], d['roofline']['phase_ms'].get('bucket'), d['verify']['mismatches'])"
echo done
