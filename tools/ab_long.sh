#!/bin/bash
# GPU check of the segmented decode's stored blocks and of the windowed sweep for streams over 65,537 bytes: the deflate parity tests, then C4-L9
# (512 x 256 KiB shard; the whole 4,096-stream set verified) with the sweep and with the chain walk,
# and the C2 headline (no change expected)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/ab_long; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_seg.py > $O/seg.log 2>&1
rc=$?; tail -2 $O/seg.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_deflate.py > $O/test.log 2>&1
rc=$?; tail -2 $O/test.log; [ $rc -eq 0 ] || exit $rc
pr() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['ms_per_step'], d['value'], d['roofline']['phase_ms'], d['verify'])" "$@"; }
for opt in match_sweep=1 match_sweep=0; do
  timeout -k 10 300 python3 bench.py --streams 512 --stream-bytes 262144 --level 9 --no-cpu-baseline --no-shard-sweep --no-e2e --option $opt > $O/l9_512_$opt.log 2>&1 || { tail -5 $O/l9_512_$opt.log; exit 1; }
  pr $O/l9_512_$opt.log "C4-L9 512 $opt"
done
timeout -k 10 300 python3 bench.py --streams 4096 --stream-bytes 262144 --level 9 --steps 3 --warmup 1 --no-cpu-baseline --no-shard-sweep --no-e2e > $O/l9_4096.log 2>&1 || { tail -5 $O/l9_4096.log; exit 1; }
pr $O/l9_4096.log "C4-L9 4096"
timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-shard-sweep --no-e2e > $O/c2.log 2>&1 || { tail -5 $O/c2.log; exit 1; }
pr $O/c2.log "C2"
