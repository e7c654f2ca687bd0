"""Debug helper: run the small deflate goldens on the GPU and list every mismatch."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "zlib-streams-ts_amd")); sys.path.insert(0, os.path.join(ROOT, "tests"))
import corpus, golden_io, oracle, zsamd
eng = zsamd.Engine(0)
cases = [(c, d) for c, d in golden_io.deflate_cases() if c["level"] >= 4]
groups = {}
for c, d in cases:
    groups.setdefault((c["level"], c["format"]), []).append((c, d))
nbad = 0
for (level, fmt), items in sorted(groups.items()):
    # also one-at-a-time to separate batching effects
    res = engine_res = eng.compress_batch_raw([d for _, d in items], fmt, level)
    for (c, d), (st, out) in zip(items, res):
        ref = oracle.compress(d, level, fmt)[1]
        if st != 1 or out != ref:
            nbad += 1
            single = eng.compress_batch_raw([d], fmt, level)[0][1]
            i = next((k for k in range(min(len(out), len(ref))) if out[k] != ref[k]), None)
            print("BAD", level, fmt, c["spec"].get("kind"), c["in_len"], "st", st, "len", len(out), len(ref),
                  "first diff", i, "single-ok", single == ref, flush=True)
print("total bad", nbad)
