"""Per-kernel SQ counters of a tools/pmc_sq.sh output directory, with the
ratios that bound an integer/LDS kernel:

  lds_bank_conflict_frac = SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE
                           (extra cycles / all LDS-array cycles, MI355X_MICROARCH.md LDS section)
  valu_busy              = 4 * SQ_INSTS_VALU / (1024 SIMDs * GRBM_GUI_ACTIVE / 8)
                           (a wave64 VALU instruction holds its SIMD 4 cycles; GRBM_GUI_ACTIVE
                           is summed over the 8 XCDs; the two come from different passes)
  active / wait / wait_inst = SQ_ACTIVE_INST_ANY, SQ_WAIT_ANY, SQ_WAIT_INST_ANY over SQ_WAVE_CYCLES
                           (disjoint; they sum to ~1)

usage: python tools/sq_summary.py DIR [kernel-substring] [--json OUT.json]"""
import collections, csv, glob, json, os, re, sys

args = [a for a in sys.argv[1:]]
out_json = None
if "--json" in args:
    i = args.index("--json")
    out_json = args[i + 1]
    del args[i:i + 2]
d = args[0]
pat = args[1] if len(args) > 1 else ""
agg = collections.defaultdict(lambda: collections.defaultdict(list))
dur = collections.defaultdict(list)
for f in sorted(glob.glob(os.path.join(d, "sq*", "run_counter_collection.csv"))):
    seen = set()
    for r in csv.DictReader(open(f)):
        full = r["Kernel_Name"].split("(")[0].replace("void ", "").replace(" ", "")
        base = re.sub(r"<[^>]*>", "", full)
        # the merged kernel and, for templates, each instance on its own
        for k in ({base, full} if full != base else {base}):
            agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
            if (f, r["Dispatch_Id"], k) not in seen:
                seen.add((f, r["Dispatch_Id"], k))
                dur[k].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))


def derived(v):
    out = {}
    if v.get("SQ_LDS_IDX_ACTIVE"):
        out["lds_bank_conflict_frac"] = v.get("SQ_LDS_BANK_CONFLICT", 0.0) / v["SQ_LDS_IDX_ACTIVE"]
    if v.get("GRBM_GUI_ACTIVE") and "SQ_INSTS_VALU" in v:
        out["valu_busy"] = 4 * v["SQ_INSTS_VALU"] / (1024 * v["GRBM_GUI_ACTIVE"] / 8)
    wc = v.get("SQ_WAVE_CYCLES")
    if wc:
        for c, name in (("SQ_ACTIVE_INST_ANY", "active"), ("SQ_WAIT_ANY", "wait"), ("SQ_WAIT_INST_ANY", "wait_inst")):
            if c in v:
                out[name + "_frac_of_wave_cycles"] = v[c] / wc
    return {k: round(x, 4) for k, x in out.items()}


res = {}
for k, cs in sorted(agg.items()):
    if pat not in k:
        continue
    v = {c: x[-1] for c, x in cs.items()}  # the last dispatch of each pass (a timed step)
    e = {"counters": v, "avg_ns": sum(dur[k]) / len(dur[k]), "dispatches": len(dur[k])}
    e.update(derived(v))
    res[k] = e
    print(k, "(avg %.3f ms over %d dispatches)" % (e["avg_ns"] / 1e6, e["dispatches"]))
    for c in sorted(v):
        print("   %-24s %16.0f" % (c, v[c]))
    for c, x in derived(v).items():
        print("   %-32s %8.4f" % (c, x))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', 'zlib-streams-ts_amd'))
import zsamd  # noqa: E402

res['_build_id'] = zsamd.build_id()  # the build these counters belong to
if out_json:
    json.dump(res, open(out_json, "w"), indent=1, sort_keys=True)
