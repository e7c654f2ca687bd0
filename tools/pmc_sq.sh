#!/bin/bash
# SQ counter pass for the deflate kernels (one rocprofv3 --pmc pass per counter group).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=$1; shift
mkdir -p "$OUT"
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY --output-format csv -d "$OUT/sq1" -o run -- python3 bench.py --no-cpu-baseline "$@" > "$OUT/sq1.log" 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_BUSY_CYCLES SQ_LDS_IDX_ACTIVE SQ_INST_CYCLES_VMEM_RD GRBM_GUI_ACTIVE --output-format csv -d "$OUT/sq2" -o run -- python3 bench.py --no-cpu-baseline "$@" > "$OUT/sq2.log" 2>&1 || exit $?
echo pmc-done
