#!/bin/bash
# rocprofv3 evidence for every BASELINE config of the current build (run through gpurun):
# kernel trace + FETCH_SIZE / WRITE_SIZE passes per config, SQ passes for the C2 and C4-L1 kernels.
# usage: tools/measure_profiles.sh OUTDIR
set -u
OUT=$1
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p "$OUT"
run() {  # name seconds command...
  local name=$1 secs=$2; shift 2
  echo "=== $name $(date +%T)"
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  tail -n 1 "$OUT/$name.log" | cut -c1-200
  if [ $rc -ne 0 ]; then echo "=== $name failed ($rc)"; exit $rc; fi
}
run p_c2 400 tools/profile.sh "$OUT/c2"
run p_c4_l1 400 tools/profile.sh "$OUT/c4_l1" --streams 512 --stream-bytes 262144 --level 1
run p_c4_l9 400 tools/profile.sh "$OUT/c4_l9" --streams 512 --stream-bytes 262144 --level 9
run p_c5_gzip 400 tools/profile.sh "$OUT/c5_gzip_l6" --format gzip --streams 1024
run p_c3 400 tools/profile.sh "$OUT/c3" --mode inflate
run p_c5_gunzip 400 tools/profile.sh "$OUT/c5_gunzip" --mode inflate --format gzip --streams 8192 --replicas 1
run p_c5_d64 400 tools/profile.sh "$OUT/c5_d64" --mode inflate --format deflate64-raw --streams 8192 --replicas 1
run sq_c2 400 tools/pmc_sq.sh "$OUT/sq_c2"
run sq_c4_l1 400 tools/pmc_sq.sh "$OUT/sq_c4_l1" --streams 512 --stream-bytes 262144 --level 1
echo measure-done
