#!/bin/bash
# Round 5: the whole GPU suite, then C5-ii (deflate64 decode, split kernels queued first on a
# high-priority stream) with its shard sweep, and a 2-rank gloo rehearsal of the decode bench
# (its step now ends with the size all-gather).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05a; mkdir -p $O
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gputests.log 2>&1
rc=$?; tail -3 $O/gputests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench.py --mode inflate --format deflate64-raw --streams 8192 --replicas 1 --no-e2e --no-cpu-baseline > $O/c5ii.log 2>&1 || { tail -5 $O/c5ii.log; exit 1; }
python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('C5-ii', d['value'], d['ms_per_step'], d.get('shard_sweep_ms'), d['roofline']['phase_ms'], d['verify'])" $O/c5ii.log
ZS_BENCH_BACKEND=gloo timeout -k 10 400 python3 bench.py --gpus 2 --mode inflate --format gzip --streams 8192 --replicas 1 --steps 5 --warmup 2 --no-cpu-baseline > $O/inflate_2ranks_gloo_1gpu.log 2>&1 || { tail -5 $O/inflate_2ranks_gloo_1gpu.log; exit 1; }
tail -1 $O/inflate_2ranks_gloo_1gpu.log | cut -c1-300
