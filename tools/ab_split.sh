#!/bin/bash
# A/B of libzsgpu.so builds on the single large deflate64 member (tools/d64_single.py): tools/ab_split.sh LIB...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for lib in "$@"; do
  echo "== $lib"
  ZS_LIB=$lib timeout -k 10 120 python3 tools/d64_single.py 2>&1 | grep -v amdgpu.ids | head -1
done
