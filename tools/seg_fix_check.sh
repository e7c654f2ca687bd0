#!/bin/bash
# GPU check of the segmented decode's end-of-block fix and bulk runs: the seg / inflate / split parity
# tests, then the C5-ii A/B (all fixtures, none, the ones the segmented decode takes)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/seg_fix; mkdir -p $O
for t in test_gpu_seg test_gpu_inflate test_gpu_split; do
  timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/$t.py > $O/$t.log 2>&1
  rc=$?; tail -2 $O/$t.log; [ $rc -eq 0 ] || exit $rc
done
C5_FIX="payload_63k payload_64k rand_block" tools/c5ii_ab.sh
