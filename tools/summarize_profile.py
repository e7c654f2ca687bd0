"""Summarize a tools/profile.sh directory into profiles/<round>/summary.json:
per kernel: calls, average duration (kernel trace), FETCH_SIZE / WRITE_SIZE
(KiB per dispatch as rocprofv3 reports them) and the HBM bytes per launch.
gfx950 FETCH_SIZE counts half of the bytes of wide coalesced reads (16 B per
lane; MI355X_MICROARCH.md, HBM), and other widths are uncalibrated: the read
side is doubled only for the kernels whose reads are of that kind (WIDE_READ);
hbm_bytes_corrected is the raw sum for every other kernel, and each entry says
which it got ("fetch_correction")."""
import collections, csv, json, os, re, sys


def knames(name):
    """'void zs_k_fast<2>(...)' -> ['zs_k_fast', 'zs_k_fast<2>']: every kernel under its
    merged name and, for templates, each instance under its own"""
    full = name.split("(")[0].replace("void ", "").replace(" ", "").strip()
    base = re.sub(r"<[^>]*>", "", full)
    return [base] if base == full else [base, full]


# kernels whose dominant reads are 16-byte-per-lane coalesced loads of the input
# (deflate_match.hip zs_k_match, deflate_sweep.hip zs_k_sweep window loads)
WIDE_READ = {"zs_k_match", "zs_k_sweep"}

src, dst = sys.argv[1], sys.argv[2]
stats = {}
for r in csv.DictReader(open(os.path.join(src, "trace", "run_kernel_stats.csv"))):
    for k in knames(r["Name"]):
        e = stats.setdefault(k, {"calls": 0, "total_ns": 0.0})
        e["calls"] += int(r["Calls"])
        e["total_ns"] += float(r["TotalDurationNs"])
        e["avg_ns"] = e["total_ns"] / e["calls"]
cnt = collections.defaultdict(lambda: collections.defaultdict(list))
for kind in ("fetch", "write"):
    p = os.path.join(src, kind, "run_counter_collection.csv")
    if not os.path.exists(p):
        continue
    for r in csv.DictReader(open(p)):
        for k in knames(r["Kernel_Name"]):
            cnt[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
out = {}
for k, v in stats.items():
    e = dict(v)
    f, w = cnt[k].get("FETCH_SIZE"), cnt[k].get("WRITE_SIZE")
    if f:
        e["fetch_kib"] = sum(f) / len(f)
    if w:
        e["write_kib"] = sum(w) / len(w)
    if f and w:
        e["hbm_bytes_raw"] = (e["fetch_kib"] + e["write_kib"]) * 1024
        wide = re.sub(r"<[^>]*>", "", k) in WIDE_READ
        e["fetch_correction"] = "x2 (16-B coalesced reads)" if wide else "none (narrow reads: uncalibrated, raw)"
        e["hbm_bytes_corrected"] = ((2 if wide else 1) * e["fetch_kib"] + e["write_kib"]) * 1024
    out[k] = e
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', 'zlib-streams-ts_amd'))
import zsamd  # noqa: E402

out['_build_id'] = zsamd.build_id()  # the build these counters belong to
os.makedirs(os.path.dirname(dst), exist_ok=True)
json.dump(out, open(dst, "w"), indent=1, sort_keys=True)
for k, e in sorted(((k, e) for k, e in out.items() if not k.startswith("_")), key=lambda kv: -kv[1]["total_ns"]):
    print("%-32s calls %3d avg %10.3f ms  hbm(raw) %s" % (k[:32], e["calls"], e["avg_ns"] / 1e6,
                                                        "%.1f MB" % (e["hbm_bytes_raw"] / 1e6) if "hbm_bytes_raw" in e else "-"))
