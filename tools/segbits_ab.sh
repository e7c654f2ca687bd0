#!/bin/bash
# A/B of seg_bits (input bits per lane of an entry's first block) on the decode configs and their 8-GPU shards
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/segbits_ab; mkdir -p $O
pr() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['ms_per_step'], {k: v for k, v in d['roofline']['phase_ms'].items() if v > 0.05})" "$@"; }
X="--no-cpu-baseline --no-e2e --no-shard-sweep"
C4D="--mode inflate --stream-bytes 262144 --streams 4096 --replicas 1 --corpus text $X"
C4S="--mode inflate --stream-bytes 262144 --streams 512 --replicas 1 --corpus text $X"
C5I="--mode inflate --format gzip --streams 8192 --replicas 1 $X"
C5S="--mode inflate --format gzip --streams 1024 --replicas 1 $X"
for b in ${SB:-2048 4096 8192}; do
  for c in C4S C5S C4D C5I; do
    timeout -k 10 300 python3 bench.py ${!c} --option seg_bits=$b > $O/${c}_$b.log 2>&1 || { tail -3 $O/${c}_$b.log; exit 1; }
    pr $O/${c}_$b.log "$c $b"
  done
done
