#!/bin/bash
# SQ counter passes for the deflate kernels (one rocprofv3 --pmc pass per counter group).
# usage: tools/pmc_sq.sh OUTDIR [bench args...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=$1; shift
mkdir -p "$OUT"
i=0
for group in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY" \
             "SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_BUSY_CYCLES SQ_LDS_IDX_ACTIVE SQ_INST_CYCLES_VMEM_RD GRBM_GUI_ACTIVE" \
             "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_ANY SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_MISC SQ_INSTS_BRANCH"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $group --output-format csv -d "$OUT/sq$i" -o run -- python3 bench.py --no-cpu-baseline --no-shard-sweep --no-e2e --no-verify --steps 2 --warmup 1 "$@" > "$OUT/sq$i.log" 2>&1 || exit $?
done
python3 tools/sq_summary.py "$OUT" zs_k_ --json "$OUT/sq_summary.json" > "$OUT/sq_summary.txt"
echo pmc-done
