#!/bin/bash
# GPU check of zs_k_fast_mr (levels 1..3 from member runs): its parity test, then C4-L1 (512 x 256 KiB shard,
# golden-checked) with fast_mr = 1 and 0
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/ab_fastmr; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_deflate.py -k "member_run or group_fast" > $O/test.log 2>&1
rc=$?; tail -3 $O/test.log; [ $rc -eq 0 ] || exit $rc
pr() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['ms_per_step'], d['value'], d['roofline']['phase_ms'], d['verify'])" "$@"; }
for opt in fast_mr=1 fast_mr=0; do
  timeout -k 10 300 python3 bench.py --streams 512 --stream-bytes 262144 --level 1 --no-cpu-baseline --no-shard-sweep --no-e2e --option $opt > $O/l1_512_$opt.log 2>&1 || { tail -5 $O/l1_512_$opt.log; exit 1; }
  pr $O/l1_512_$opt.log "C4-L1 512 $opt"
done
