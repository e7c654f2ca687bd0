#!/bin/bash
# Decode configs with their 8-GPU shard (what rank 0 decodes) and its phases: 4,096 x 256 KiB L6 (512-member
# shard), C5-i gunzip (1,024), C5-ii deflate64 (1,025); extra bench arguments pass through (--option ...)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/dec_shards${TAG:+_$TAG}; mkdir -p $O
pr() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['ms_per_step'], d['shard_sweep_ms'], d.get('shard8_phase_ms'))" "$@"; }
X="--no-cpu-baseline --no-e2e --steps 10 --warmup 3 $*"
timeout -k 10 300 python3 bench.py --mode inflate --stream-bytes 262144 --streams 4096 --replicas 1 --corpus text $X > $O/c4.log 2>&1 || { tail -5 $O/c4.log; exit 1; }
pr $O/c4.log "C4dec"
timeout -k 10 300 python3 bench.py --mode inflate --format gzip --streams 8192 --replicas 1 $X > $O/c5i.log 2>&1 || { tail -5 $O/c5i.log; exit 1; }
pr $O/c5i.log "C5-i"
timeout -k 10 300 python3 bench.py --mode inflate --format deflate64-raw --streams 8192 --replicas 1 $X > $O/c5ii.log 2>&1 || { tail -5 $O/c5ii.log; exit 1; }
pr $O/c5ii.log "C5-ii"
