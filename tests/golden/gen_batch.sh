#!/bin/bash
# Generates per-stream (u32 len, sha256[:16]) goldens for the SURVEY.md §8(d)
# batch sets with the reference bundle, 8 node processes per set.
set -e
cd "$(dirname "$0")"
for SET in "$@"; do
  pids=()
  for P in 0 1 2 3 4 5 6 7; do node gen_golden.mjs batch "$SET" 8 "$P" & pids+=($!); done
  for p in "${pids[@]}"; do wait "$p"; done
  cat /tmp/golden_${SET}_{0,1,2,3,4,5,6,7}.bin > "batch_${SET}.bin"
  rm -f /tmp/golden_${SET}_*.bin
  echo "done $SET $(stat -c %s batch_${SET}.bin)"
done
