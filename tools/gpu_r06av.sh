#!/bin/bash
# round 6: the sweep's next group's records read with this group's (vs only its last key)
set -o pipefail
O=gpurun_out/r06av; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_deflate.py -x -q --timeout 300 --timeout-method thread > $O/test.log 2>&1 || { tail -30 $O/test.log; exit 1; }
tail -1 $O/test.log
X="--steps 10 --warmup 3 --no-cpu-baseline --no-e2e --no-shard-sweep"
for v in default ab0 default ab0; do
  if [ $v = default ]; then L=""; else L=variants/$v/libzsgpu.so; fi
  ZS_LIB=$L timeout -k 10 300 python bench.py $X > $O/c2_$v.log 2>&1 || exit 1
  python3 -c "import json; d=json.loads(open('$O/c2_$v.log').read().strip().splitlines()[-1]); print('c2 $v', d['ms_per_step'], d['roofline']['phase_ms']['sweep'], d['verify']['mismatches'])"
  ZS_LIB=$L timeout -k 10 300 python bench.py $X --streams 512 --stream-bytes 262144 --level 9 > $O/l9_$v.log 2>&1 || exit 1
  python3 -c "import json; d=json.loads(open('$O/l9_$v.log').read().strip().splitlines()[-1]); print('l9 $v', d['ms_per_step'], d['roofline']['phase_ms']['sweep'], d['verify']['mismatches'])"
done
echo done
