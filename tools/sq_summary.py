"""Print per-kernel SQ counters of a tools/pmc_sq.sh output directory, with
per-wave-instruction ratios.  usage: python tools/sq_summary.py DIR [kernel-substring]"""
import collections, csv, glob, os, sys

d = sys.argv[1]
pat = sys.argv[2] if len(sys.argv) > 2 else ""
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(os.path.join(d, "sq*", "run_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        agg[r["Kernel_Name"].split("(")[0]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in sorted(agg.items()):
    if pat not in k:
        continue
    v = {c: x[-1] for c, x in cs.items()}
    print(k)
    for c in sorted(v):
        print("   %-24s %16.0f" % (c, v[c]))
    wc = v.get("SQ_WAVE_CYCLES")
    if wc:
        for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
            if c in v:
                print("   %-24s %6.1f%% of wave cycles" % (c, 100 * v[c] / wc))
