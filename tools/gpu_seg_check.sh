#!/bin/bash
# The segmented decode's GPU checks and shard-size bench lines (gpurun).
# usage: tools/gpu_seg_check.sh OUTDIR [bench options...]
set -u
OUT=$1; shift
mkdir -p "$OUT"
T="timeout -k 10"
$T 600 python3 -u -m pytest tests/test_gpu_seg.py tests/test_gpu_inflate.py tests/test_gpu_split.py tests/test_gpu_boundary.py -m gpu -x -v --timeout 200 --timeout-method thread > "$OUT/tests.log" 2>&1
rc=$?; tail -3 "$OUT/tests.log"; [ $rc -eq 0 ] || exit $rc
C4D="--mode inflate --stream-bytes 262144 --replicas 1 --corpus text --no-shard-sweep --no-e2e --no-cpu-baseline"
C5I="--mode inflate --format gzip --replicas 1 --no-shard-sweep --no-e2e --no-cpu-baseline"
C5D="--mode inflate --format deflate64-raw --replicas 1 --no-shard-sweep --no-e2e --no-cpu-baseline"
for n in 512 4096; do $T 200 python3 bench.py $C4D --streams $n "$@" > "$OUT/c4d_$n.log" 2>&1 || exit 1; done
for n in 1024 8192; do $T 200 python3 bench.py $C5I --streams $n "$@" > "$OUT/c5i_$n.log" 2>&1 || exit 1; done
for n in 1024 8192; do $T 200 python3 bench.py $C5D --streams $n "$@" > "$OUT/c5d_$n.log" 2>&1 || exit 1; done
for f in "$OUT"/c*.log; do python3 - "$f" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().split("\n")[-1])
print(sys.argv[1].split("/")[-1], d["ms_per_step"], {k: v for k, v in d["roofline"]["phase_ms"].items() if v > 0.05})
PY
done
