#!/bin/bash
# Copies a tools/measure_r06.sh output directory's bench lines and summaries into profiles/r06/.
# usage: tools/collect_r06.sh OUTDIR
set -eu
SRC=$1
DST=$(dirname "$0")/../profiles/r06
mkdir -p "$DST/bench"
for f in "$SRC"/c*.log; do [ -f "$f" ] && tail -n 1 "$f" > "$DST/bench/$(basename "${f%.log}").json"; done
[ -f "$SRC/gputest.log" ] && cp "$SRC/gputest.log" "$DST/gputest_final.log"
for d in "$SRC"/prof_*; do
  [ -d "$d" ] || continue
  t=${d##*/prof_}
  [ -f "$d/summary.json" ] && cp "$d/summary.json" "$DST/summary_$t.json"
  [ -f "$d/trace/run_kernel_stats.csv" ] && cp "$d/trace/run_kernel_stats.csv" "$DST/kernel_stats_$t.csv"
done
for d in "$SRC"/sq_*; do
  [ -d "$d" ] || continue
  t=${d##*/sq_}
  [ -f "$d/sq_summary.json" ] && cp "$d/sq_summary.json" "$DST/sq_summary_$t.json"
  [ -f "$d/sq_summary.txt" ] && cp "$d/sq_summary.txt" "$DST/sq_summary_$t.txt"
done
ls "$DST"
for f in smoke bench_2ranks_gloo_1gpu inflate_2ranks_gloo_1gpu; do
  [ -f "$SRC/$f.log" ] && cp "$SRC/$f.log" "$DST/$f.log"
done
true
