#!/bin/bash
# A/B of seg_big_bits (members with more input bits also walk from the finder's block starts): the C4
# decode (4,096 x 256 KiB T-corpus), its 8-GPU shard (512 members), C5-i gunzip and C5-ii
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/big_ab; mkdir -p $O
pr() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['ms_per_step'], {k: v for k, v in d['roofline']['phase_ms'].items() if v > 0.05})" "$@"; }
C4D="--mode inflate --stream-bytes 262144 --streams 4096 --replicas 1 --corpus text --no-cpu-baseline --no-e2e --no-shard-sweep"
C4S="--mode inflate --stream-bytes 262144 --streams 512 --replicas 1 --corpus text --no-cpu-baseline --no-e2e --no-shard-sweep"
C5I="--mode inflate --format gzip --streams 8192 --replicas 1 --no-cpu-baseline --no-e2e --no-shard-sweep"
for b in ${BIG:-2097152 524288 262144 131072}; do
  for c in C4D C4S C5I; do
    timeout -k 10 300 python3 bench.py ${!c} --option seg_big_bits=$b > $O/${c}_$b.log 2>&1 || { tail -3 $O/${c}_$b.log; exit 1; }
    pr $O/${c}_$b.log "$c $b"
  done
done
