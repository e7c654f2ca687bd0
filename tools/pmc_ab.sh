#!/bin/bash
# SQ counters for two library variants: tools/pmc_ab.sh OUTDIR LIB_A LIB_B [bench args]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$1; A=$2; B=$3; shift 3
ZS_LIB=$A tools/pmc_sq.sh "$OUT/a" "$@" && ZS_LIB=$B tools/pmc_sq.sh "$OUT/b" "$@"
