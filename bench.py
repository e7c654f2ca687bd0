#!/usr/bin/env python3
"""Headline benchmark: uncompressed MB/s, deflate-raw L6, one 4096 x 64 KiB
synthetic T-corpus batch (BASELINE.json configs[1]) at 1/2/4/8 GPUs.

One process per GPU: for N > 1 either a launcher's ranks (torch.distributed.run
sets WORLD_SIZE; it must equal --gpus) or, run directly with --gpus N, N child
ranks this script starts itself before any GPU call.  A "step" is one batch
compression, inputs already resident in HBM, outputs written to HBM.

* Strong scaling (default, the north star's "batch partitioned across the
  GPUs"): the ONE global batch of --streams streams is split into contiguous
  shards, rank r compressing streams shard_range(S, N, r) (zsamd/shard.py).
  value = global input bytes / max-over-ranks step time.
* --scaling weak: every rank compresses its own --streams streams.
* For N > 1 every step ends with the final per-stream size all-gather over
  RCCL (the only collective: it gives every rank the global output layout).

After the timed region, outside it: every output stream is checked against
the committed reference golden of the workload (tests/golden/batch_*.bin,
made by the reference bundle) -- a mismatch fails the run; --no-verify skips
it (profiling runs only).  On rank 0 at N=1 the line also carries the shard
sweep (the step time of the 512 / 1024 / 2048-stream shards a rank gets at
8 / 4 / 2 GPUs), the end-to-end host->host rate through zs_deflate_batch, and
the CPU baselines.  --mode inflate decodes members (C3; with --format gzip the
C5-i gunzip; with --format deflate64-raw the C5-ii deflate64 decode).

Prints ONE JSON line on rank 0.  See DESIGN.md "Measurement".
"""
import argparse
import ctypes
import hashlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "zlib-streams-ts_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s peak
# SURVEY.md section 6 (measured in the survey container: Intel Xeon 8 vCPU,
# Node v12.22.9, the reference's own dist/ bundle, median of 3 after warm-up).
# The reference tree does not exist on the GPU box, so it cannot be re-timed there.
REFERENCE_TS = {
    "deflate": {"value": 2.57, "cores": 1, "value_8_cores": 20.2},
    "deflate-l1-256k": {"value": 4.82, "cores": 1},
    "deflate-l9-256k": {"value": 2.10, "cores": 1},
    "inflate": {"value": 84.2, "cores": 1},
    "gunzip": {"value": 80.3, "cores": 1},
    "deflate64": {"value": 17.9, "cores": 1},
}
GOLDENS = {("text", 65536, 6, "deflate-raw"): "t64_l6_raw", ("text", 65536, 6, "gzip"): "t64_l6_gzip",
           ("text", 262144, 1, "deflate-raw"): "t256_l1_raw", ("text", 262144, 9, "deflate-raw"): "t256_l9_raw",
           ("mixed", 65536, 6, "deflate-raw"): "m64_l6_raw", ("text", 262144, 6, "deflate-raw"): "t256_l6_raw"}
# what the reference's DecompressionStream returns for those streams (where its
# window-wrap copy, inffast.ts:133-147, makes that differ from the source)
GOLDENS_DEC = {("text", 262144, 6, "deflate-raw"): "t256_l6_raw_dec"}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--streams", type=int, default=4096, help="global batch (strong) or per-GPU batch (weak)")
    ap.add_argument("--stream-bytes", type=int, default=65536)
    ap.add_argument("--level", type=int, default=6)
    ap.add_argument("--format", default="deflate-raw")
    ap.add_argument("--corpus", default=None,
                    help="text | mixed | rand (default: text; mixed for the C3 deflate-raw inflate mode)")
    ap.add_argument("--scaling", default="strong", choices=["strong", "weak"])
    ap.add_argument("--cpu-seconds", type=float, default=8.0, help="bounded CPU-baseline sample (per variant)")
    ap.add_argument("--cpu-threads", type=int, default=8)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-verify", action="store_true", help="skip the golden check (profiling runs only)")
    ap.add_argument("--no-shard-sweep", action="store_true")
    ap.add_argument("--no-e2e", action="store_true")
    ap.add_argument("--mode", default="deflate", choices=["deflate", "inflate"],
                    help="deflate: the headline (configs[1]); inflate: decode of pre-built members (configs[2], C5)")
    ap.add_argument("--replicas", type=int, default=16, help="inflate: members = streams x replicas (C3: 4096 x 16)")
    ap.add_argument("--no-fixtures", action="store_true", help="deflate64-raw: without the reference's fixtures (A/B only)")
    ap.add_argument("--fixtures", default="", help="deflate64-raw: only the fixtures whose names contain one of these "
                    "comma-separated strings (A/B only)")
    ap.add_argument("--option", action="append", default=[], metavar="NAME=VALUE",
                    help="engine option (zs_set_option), e.g. lane_block=16; repeatable")
    return ap.parse_args()


def set_options(eng, args):
    for o in args.option:
        k, v = o.split("=")
        eng.set_option(k, int(v))


class Dist:
    """torch.distributed plumbing: one process per GPU (RCCL), or a single process."""

    def __init__(self):
        import torch
        import torch.distributed as dist

        self.torch, self.dist = torch, dist
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local = int(os.environ.get("LOCAL_RANK", "0"))
        # ZS_BENCH_BACKEND=gloo + more ranks than GPUs: a functional rehearsal of the multi-rank path on a
        # one-GPU box (ranks share the device); the driver's runs use RCCL, one rank per GPU
        backend = os.environ.get("ZS_BENCH_BACKEND", "nccl")
        if backend != "nccl":
            self.local %= max(1, torch.cuda.device_count())
        if self.world > 1:
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            if backend == "nccl":
                dist.init_process_group("nccl", device_id=torch.device("cuda", self.local))
            else:
                dist.init_process_group(backend)
        torch.cuda.set_device(self.local)
        self.dev = torch.device("cuda", self.local)

    def barrier(self):
        self.torch.cuda.synchronize()
        if self.world > 1:
            self.dist.barrier()
        self.torch.cuda.synchronize()

    def max(self, x):
        t = self.torch.tensor([float(x)], dtype=self.torch.float64, device=self.dev)
        if self.world > 1:
            self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t.item())

    def sum(self, x):
        t = self.torch.tensor([int(x)], dtype=self.torch.int64, device=self.dev)
        if self.world > 1:
            self.dist.all_reduce(t)
        return int(t.item())

    def close(self):
        if self.world > 1:
            self.dist.destroy_process_group()


def profile_tag(args):
    """The config name the committed profiles carry (profiles/<round>/summary_<tag>.json)."""
    if args.mode == "inflate":
        if args.format == "deflate-raw" and args.stream_bytes == 262144:
            return "c4_decode"  # the 4096 x 256 KiB members decoded back
        return {"gzip": "c5_gunzip", "deflate64-raw": "c5_d64"}.get(args.format, "c3")
    if args.format == "gzip":
        return "c5_gzip_l%d" % args.level
    return "c2" if args.stream_bytes == 65536 else "c4_l%d" % args.level


def _tagged_first(files, tag):
    """Only the files of this config (name contains _<tag>.): another config's launches of the same kernel are
    other launches (C5-ii's walk once matched C5-i's duration and borrowed its traffic)."""
    if not tag:
        return files
    return [f for f in files if ("_%s." % tag) in os.path.basename(f)]


def build_id():
    import zsamd
    return zsamd.build_id()


def profiled_traffic(kernel, kernel_ms, tag=None):
    """`kernel`: a name or a list of names (template instances) tried in each file in turn."""
    names = [kernel] if isinstance(kernel, str) else list(kernel)
    return _profiled_traffic(names, kernel_ms, tag)


def _profiled_traffic(names, kernel_ms, tag=None):
    """HBM bytes per launch of `kernel` from the newest committed rocprofv3
    summary (profiles/*/summary*.json: FETCH_SIZE / WRITE_SIZE passes, gfx950
    read correction by tools/summarize_profile.py) -- used only when that
    profile was made from this build (its "_build_id", zsamd.build_id()) and its
    average kernel duration agrees with this run's HIP-event time within 10 %;
    otherwise (None, reason)."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "*", "summary*.json")))  # round directories sort in order
    files = _tagged_first(files, tag)
    stale = None
    bid = build_id()
    for f in reversed(files):  # this config's files first, newest round first; the first matching duration
        try:
            j = json.load(open(f))
        except (OSError, ValueError):
            continue
        src = os.path.relpath(f, ROOT)
        for kernel in names:
            e = j.get(kernel)
            if not e or "hbm_bytes_corrected" not in e:
                continue
            if j.get("_build_id") != bid:
                stale = stale or "stale: %s is of build %s, this is build %s" % (src, j.get("_build_id"), bid)
                continue
            prof_ms = e["avg_ns"] / 1e6
            if abs(prof_ms - kernel_ms) > 0.1 * kernel_ms:
                stale = stale or "stale: %s has %s at %.3f ms, this run %.3f ms" % (src, kernel, prof_ms, kernel_ms)
                continue
            return int(e["hbm_bytes_corrected"]), "%s (%s avg %.3f ms)" % (src, kernel, prof_ms)
    return None, stale or "no committed profile for %s" % " / ".join(names)


def profiled_ceilings(kernel, kernel_ms, tag=None):
    """`kernel`: a name or a list of names (template instances) tried in each file in turn."""
    names = [kernel] if isinstance(kernel, str) else list(kernel)
    return _profiled_ceilings(names, kernel_ms, tag)


def _profiled_ceilings(names, kernel_ms, tag=None):
    """The SQ-counter ratios that bound `kernel` below the HBM roofline, from the
    newest committed tools/pmc_sq.sh summary (profiles/*/sq_summary*.json,
    written by tools/sq_summary.py --json): LDS bank-conflict cycles over LDS
    cycles, VALU busy over SIMD-cycles, and the active / parked / issue-stalled
    split of wave cycles.  Used only when that profile's kernel duration agrees
    with this run's within 15 % (counter passes run a little slower)."""
    import glob

    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "*", "sq_summary*.json")) +
                   glob.glob(os.path.join(ROOT, "profiles", "*", "*", "sq_summary*.json")))
    files = _tagged_first(files, tag)
    stale = None
    bid = build_id()
    for f in reversed(files):  # this config's files first, newest round first; the first matching duration
        try:
            j = json.load(open(f))
        except (OSError, ValueError):
            continue
        src = os.path.relpath(f, ROOT)
        for kernel in names:
            e = j.get(kernel)
            if not e:
                continue
            if j.get("_build_id") != bid:
                stale = stale or "stale: %s is of build %s, this is build %s" % (src, j.get("_build_id"), bid)
                continue
            prof_ms = e["avg_ns"] / 1e6
            if abs(prof_ms - kernel_ms) > 0.15 * kernel_ms:
                stale = stale or "stale: %s has %s at %.3f ms, this run %.3f ms" % (src, kernel, prof_ms, kernel_ms)
                continue
            out = {k: e[k] for k in ("lds_bank_conflict_frac", "valu_busy", "active_frac_of_wave_cycles",
                                     "wait_frac_of_wave_cycles", "wait_inst_frac_of_wave_cycles") if k in e}
            out["source"] = "%s (%s avg %.3f ms under --pmc)" % (src, kernel, prof_ms)
            return out
    return {"source": stale or "no committed SQ summary for %s" % " / ".join(names)}


def timed_port(fn, items, seconds, threads):
    """Runs fn(item) over items until `seconds` of wall time pass; returns
    (items done, wall seconds).  The oracle is a ctypes C library, so threads
    run in parallel (ctypes releases the GIL)."""
    from concurrent.futures import ThreadPoolExecutor

    done, t0 = 0, time.perf_counter()
    if threads == 1:
        for it in items:
            fn(it)
            done += 1
            if time.perf_counter() - t0 >= seconds:
                break
        return done, time.perf_counter() - t0
    with ThreadPoolExecutor(threads) as ex:
        k = 0
        while k < len(items) and time.perf_counter() - t0 < seconds:
            batch = items[k:k + 4 * threads]
            list(ex.map(fn, batch))
            done += len(batch)
            k += len(batch)
    return done, time.perf_counter() - t0


def cpu_baseline(args, kind, make_item, fn, unit_bytes, n_items, ref_key):
    """The C oracle (oracle/, a restatement of the reference algorithm; kind
    "port") on a bounded sample of the same workload on this host, 1 thread and
    --cpu-threads threads; the reference TS figure is quoted with provenance."""
    import oracle

    oracle.lib()
    items = [make_item(i) for i in range(min(n_items, 4096))]
    fn(items[0])  # warm
    k1, t1 = timed_port(fn, items, args.cpu_seconds, 1)
    kp, tp = timed_port(fn, items, args.cpu_seconds, args.cpu_threads)
    ref = REFERENCE_TS.get(ref_key)
    out = {"value": round(k1 * unit_bytes / t1 / 1e6, 3), "unit": "MB/s", "cores": 1, "kind": "port",
           "sample": "%d %s units of %d B (of the workload's %d), oracle/ C restatement, 1 thread, %.1f s"
                     % (k1, kind, unit_bytes, n_items, t1),
           "port_parallel": {"value": round(kp * unit_bytes / tp / 1e6, 3), "cores": args.cpu_threads,
                             "sample": "%d units, %.1f s" % (kp, tp)}}
    if ref:
        out["reference_ts"] = dict(ref, unit="MB/s", kind="reference",
                                   provenance="SURVEY.md section 6: the reference's dist/ bundle under Node v12.22.9 on "
                                              "the survey container's Intel Xeon (8 vCPU), median of 3 after warm-up; "
                                              "/root/reference does not exist on the GPU box, so it is quoted, not re-timed")
    return out


def layout(S, L, cap):
    in_off = (ctypes.c_uint64 * max(1, S))(*[i * L for i in range(S)])
    in_len = (ctypes.c_uint32 * max(1, S))(*([L] * S))
    out_off = (ctypes.c_uint64 * max(1, S))(*[i * cap for i in range(S)])
    out_cap = (ctypes.c_uint32 * max(1, S))(*([cap] * S))
    return in_off, in_len, out_off, out_cap


def launch_ranks(args):
    """`--gpus N` (N > 1) run directly, without a launcher's WORLD_SIZE: start the N
    ranks here -- fresh child processes, one per GPU, nothing of the GPU touched in
    this parent -- with torch.distributed's env rendezvous on 127.0.0.1, and exit
    with the first failing rank's code (the others are stopped then)."""
    import socket
    import subprocess

    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    procs = []
    for r in range(args.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(args.gpus),
                   LOCAL_WORLD_SIZE=str(args.gpus), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rc = 0
    while procs:
        for p in list(procs):
            code = p.poll()
            if code is None:
                continue
            procs.remove(p)
            if code != 0 and rc == 0:
                rc = code
                for q in procs:
                    q.terminate()
        time.sleep(0.05)
    sys.exit(rc)


def main():
    args = parse()
    world = os.environ.get("WORLD_SIZE")
    if world is None and args.gpus > 1:
        return launch_ranks(args)
    if world is not None:
        assert int(world) == args.gpus, "WORLD_SIZE=%s but --gpus %d" % (world, args.gpus)
    if args.corpus is None:
        args.corpus = "mixed" if (args.mode == "inflate" and args.format == "deflate-raw") else "text"
    if args.mode == "inflate":
        return main_inflate(args)
    import zsamd
    import zsamd.shard as shard

    D = Dist()
    torch = D.torch
    S_glob = args.streams * (D.world if args.scaling == "weak" else 1)
    lo, hi = shard.shard_range(S_glob, D.world, D.rank)
    S, L = hi - lo, args.stream_bytes
    host = zsamd.corpus(args.corpus, lo, S, L, threads=8)
    d_in = torch.frombuffer(host, dtype=torch.uint8).to(D.dev)
    cap = zsamd.deflate_capacity(L, args.format)
    d_out = torch.zeros(S * cap, dtype=torch.uint8, device=D.dev)
    d_status = torch.zeros(S, dtype=torch.int32, device=D.dev)
    d_len = torch.zeros(S, dtype=torch.int32, device=D.dev)
    in_off, in_len, out_off, out_cap = layout(S, L, cap)
    eng = zsamd.Engine(D.local)
    set_options(eng, args)
    stream = torch.cuda.current_stream(D.dev)

    def run(n):
        eng.compress_device(args.level, args.format, n, d_in.data_ptr(), in_off, in_len, d_out.data_ptr(), out_off,
                            out_cap, d_status.data_ptr(), d_len.data_ptr(), stream.cuda_stream)

    def step():
        run(S)
        if D.world > 1:
            # the final size gather (RCCL all_gather over xGMI): global output layout on every rank
            sizes = shard.gather_sizes(d_len, S_glob)
            shard.global_offsets(sizes)

    for _ in range(args.warmup):
        step()
    D.barrier()
    eng.set_timing(True)
    phases = {}
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()  # back to back: the phase events are read after the timed region
    D.barrier()
    elapsed = time.perf_counter() - t0
    for ph in ("checksum", "bucket", "prev", "sweep", "match", "stored", "fast", "parse", "trees", "layout", "emit",
               "finish"):
        v = eng.last_ms(ph)  # summed over the timed steps
        if v >= 0:
            phases[ph] = phases.get(ph, 0.0) + v
    eng.set_timing(False)
    elapsed = D.max(elapsed)

    status = d_status.cpu()
    lens = d_len.cpu()
    assert int((status != 1).sum()) == 0, "some streams failed: %s" % status.unique()
    out_local = int(lens.sum())
    out_total = D.sum(out_local)
    in_total = S_glob * L

    # parity: every stream against the reference golden (outside the timed region)
    verify = {"golden": None, "checked": 0, "mismatches": 0}
    gname = GOLDENS.get((args.corpus, L, args.level, args.format))
    if not args.no_verify and gname:
        import golden_io
        recs = golden_io.batch(gname)
        ob = d_out.cpu().numpy()
        bad = checked = 0
        for i in range(S):
            if lo + i >= len(recs):
                break
            o = ob[i * cap: i * cap + int(lens[i])].tobytes()
            checked += 1
            bad += (len(o), hashlib.sha256(o).digest()[:16]) != recs[lo + i]
        verify = {"golden": "tests/golden/batch_%s.bin" % gname, "checked": D.sum(checked),
                  "mismatches": D.sum(bad)}
        assert verify["mismatches"] == 0, "outputs differ from the reference golden: %s" % verify
    elif args.no_verify:
        verify["golden"] = "skipped (--no-verify)"

    extra = {}
    if D.world == 1 and D.rank == 0:
        if not args.no_shard_sweep and args.scaling == "strong":
            # what each rank computes at 8 / 4 / 2 GPUs (same streams, one GPU)
            sweep = {}
            for m in (512, 1024, 2048):
                if m >= S:
                    continue
                run(m)
                torch.cuda.synchronize()
                t1 = time.perf_counter()
                for _ in range(args.steps):
                    run(m)
                torch.cuda.synchronize()
                sweep[str(m)] = round((time.perf_counter() - t1) / args.steps * 1e3, 4)
            sweep[str(S)] = round(elapsed / args.steps * 1e3, 4)
            extra["shard_sweep_ms"] = sweep
            if "512" in sweep:
                extra["implied_1_to_8_speedup"] = round(sweep[str(S)] / sweep["512"], 3)
        if not args.no_e2e:
            # end-to-end: caller-owned host buffers -> host buffers through zs_deflate_batch
            import numpy as np
            hout = np.zeros(S * cap, dtype=np.uint8)
            st = (ctypes.c_int32 * S)()
            ol = (ctypes.c_uint32 * S)()
            hin_ptr = ctypes.addressof((ctypes.c_char * len(host)).from_buffer(host))

            def e2e():
                eng.compress_host(args.level, args.format, S, hin_ptr, in_off, in_len, hout.ctypes.data, out_off,
                                  out_cap, st, ol)
            e2e()
            t1 = time.perf_counter()
            reps = max(1, min(args.steps, 5))
            for _ in range(reps):
                e2e()
            te = (time.perf_counter() - t1) / reps
            ok = sum(ol) == out_local and all(st[i] == 1 for i in range(S))
            extra["end_to_end"] = {"value": round(in_total / te / 1e6, 2), "unit": "MB/s", "ms": round(te * 1e3, 3),
                                   "path": "host buffers -> zs_deflate_batch (pinned staging, chunks whose copies "
                                           "overlap the kernels, device compaction) -> host buffers",
                                   "matches_device_path": bool(ok)}

    if D.rank == 0:
        ms_per_step = elapsed / args.steps * 1e3
        value = in_total / (elapsed / args.steps) / 1e6
        phase_avg = {k: round(v / args.steps, 4) for k, v in phases.items()}
        # the dominant KERNEL phase (inflate_join is the caller's stream waiting for the side stream)
        dom = max((k for k in phase_avg if k not in ("inflate_join", "finish")), key=phase_avg.get) if phase_avg else None
        roof = None
        if dom:
            # bytes_in + bytes_out per stream x streams per launch (this rank's shard)
            alg = S * L + out_local
            achieved = alg / (phase_avg[dom] / 1e3) / 1e9
            traffic, tsrc = profiled_traffic("zs_k_" + dom, phase_avg[dom], profile_tag(args))
            roof = {"bound": "hbm", "kernel": "zs_k_" + dom, "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS,
                    "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": traffic,
                    "traffic_source": tsrc, "algorithmic_bytes": alg, "kernel_ms": phase_avg[dom],
                    "phase_ms": phase_avg, "pipeline_ms": round(sum(phase_avg.values()), 4),
                    "ceilings": profiled_ceilings("zs_k_" + dom, phase_avg[dom], profile_tag(args))}
        cpu = None
        if not (args.no_cpu_baseline or D.world > 1):
            import oracle
            key = "deflate" if L == 65536 else "deflate-l%d-256k" % args.level
            cpu = cpu_baseline(args, "stream", lambda i: bytes(host[i * L:(i + 1) * L]),
                               lambda d: oracle.compress(d, args.level, args.format), L, S, key)
        line = {
            "metric": "uncompressed MB/s, deflate-raw L6, 4096x64KiB batch at 1/2/4/8 GPUs"
            if (args.format, args.level, L, args.corpus) == ("deflate-raw", 6, 65536, "text")
            else "uncompressed MB/s, %s L%d, %dx%dB %s batch" % (args.format, args.level, S_glob, L, args.corpus),
            "value": round(value, 2), "unit": "MB/s", "n_gpus": D.world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4), "higher_is_better": True, "scaling": args.scaling,
            "vs_baseline": None, "dtype": "u8", "data": "synthetic",
            "config": {"workload": "%d x %d B %s-corpus streams%s, %s level %d" % (
                S_glob, L, args.corpus, " split across the GPUs" if args.scaling == "strong" else " (per GPU x N)",
                args.format, args.level),
                "global_streams": S_glob, "streams_per_gpu": S, "stream_bytes": L, "level": args.level,
                "format": args.format, "compressed_bytes": out_total, "ratio": round(in_total / max(1, out_total), 4),
                "parallelism": "dp%d" % D.world},
            "verify": verify, "roofline": roof, "cpu_baseline": cpu,
        }
        line.update(extra)
        print(json.dumps(line), flush=True)
    D.close()


def d64_fixtures(only=""):
    """The reference's test/data deflate64 fixtures (tests/golden/d64) with their
    decoded sizes / digests from inflate_small.json (only: comma-separated name parts to keep)."""
    g = json.load(open(os.path.join(ROOT, "tests", "golden", "inflate_small.json")))
    keep = [k for k in only.split(",") if k]
    out = []
    for c in g["cases"]:
        if keep and not any(k in c["name"] for k in keep):
            continue
        if c["name"].startswith("d64_") and c.get("ok"):
            out.append((open(os.path.join(ROOT, "tests", "golden", "d64", c["name"][4:]), "rb").read(),
                        c["out_len"], c["out_sha256"]))
    return out


PHASES_INFLATE = ("inflate_lane", "inflate_long", "inflate_wave", "inflate_large", "split_find", "split_decode",
                  "split_resolve", "seg_find", "seg_walk", "seg_plan", "seg_decode", "seg_resolve", "seg_fallback",
                  "inflate_join", "inflate_check", "inflate", "finish")


def main_inflate(args):
    """Decode of pre-built members, strong scaling over the global member list.
    C3: 4096 unique M-corpus 64 KiB buffers compressed at
    deflate-raw L6 by this engine (checked against the reference batch golden),
    x16 = 65,536 members.  --format gzip: C5-i gunzip (CRC-32 trailer checked).
    --format deflate64-raw: C5-ii, the T-corpus raw-L6 streams decoded as
    deflate64 (valid deflate64: no length-258 match) with the
    reference's deflate64 fixtures interleaved.  Metric: output MB/s."""
    import zsamd
    import zsamd.shard as shard

    D = Dist()
    torch = D.torch
    S, L, R = args.streams, args.stream_bytes, args.replicas
    dec_fmt = args.format
    enc_fmt = "deflate-raw" if dec_fmt == "deflate64-raw" else dec_fmt
    eng = zsamd.Engine(D.local)
    set_options(eng, args)
    N_glob = S * R
    # the global member list: the corpus members, with (C5-ii) the reference's deflate64 fixtures
    # interleaved at fixed places -- sharded as one list, so each fixture is decoded by exactly one rank
    fx = d64_fixtures(args.fixtures) if dec_fmt == "deflate64-raw" and not args.no_fixtures else []
    gstep = max(1, N_glob // max(1, len(fx)))
    entries = []
    for i in range(N_glob):
        if fx and i % gstep == gstep // 2 and i // gstep < len(fx):
            entries.append(("f", i // gstep))
        entries.append(("u", i))
    lo, hi = shard.shard_range(len(entries), D.world, D.rank)
    mine = entries[lo:hi]
    uniq = sorted({e[1] % S for e in mine if e[0] == "u"})
    umap = {u: k for k, u in enumerate(uniq)}
    host = bytearray()
    for u in uniq:
        host += zsamd.corpus(args.corpus, u, 1, L, threads=1)
    comp = eng.compress_batch([bytes(host[k * L:(k + 1) * L]) for k in range(len(uniq))], enc_fmt, 6)
    gname = GOLDENS.get((args.corpus, L, 6, enc_fmt))
    members_checked = 0
    if gname and not args.no_verify:
        import golden_io
        recs = golden_io.batch(gname)
        for k, u in enumerate(uniq):
            if u < len(recs):
                assert (len(comp[k]), hashlib.sha256(comp[k]).digest()[:16]) == recs[u], "member source %d" % u
                members_checked += 1
    # (the fixtures: distances > 32 KiB, codes 30/31)
    members = [comp[umap[e[1] % S]] if e[0] == "u" else fx[e[1]][0] for e in mine]
    expect = [("u", umap[e[1] % S]) if e[0] == "u" else ("f", fx[e[1]][1], fx[e[1]][2]) for e in mine]
    N = len(members)
    caps = [L if e[0] == "u" else ((e[1] + 3) & ~3) for e in expect]
    blob = b"".join(members)
    d_in = torch.frombuffer(bytearray(blob), dtype=torch.uint8).to(D.dev)
    offs, o = [], 0
    for m in members:
        offs.append(o)
        o += len(m)
    oo, ooffs = 0, []
    for c in caps:
        ooffs.append(oo)
        oo += c
    in_off = (ctypes.c_uint64 * N)(*offs)
    in_len = (ctypes.c_uint32 * N)(*[len(m) for m in members])
    d_out = torch.zeros(oo, dtype=torch.uint8, device=D.dev)
    out_off = (ctypes.c_uint64 * N)(*ooffs)
    out_cap = (ctypes.c_uint32 * N)(*caps)
    i32 = lambda: torch.zeros(N, dtype=torch.int32, device=D.dev)
    d_status, d_phase, d_msg, d_len, d_cons = i32(), i32(), i32(), i32(), i32()
    stream = torch.cuda.current_stream(D.dev)

    N_all = len(entries)

    def step():
        eng.decompress_device(dec_fmt, N, d_in.data_ptr(), in_off, in_len, d_out.data_ptr(), out_off, out_cap,
                              d_status.data_ptr(), d_phase.data_ptr(), d_msg.data_ptr(), d_len.data_ptr(),
                              d_cons.data_ptr(), stream.cuda_stream)
        if D.world > 1:
            # the final size gather (RCCL all_gather over xGMI), as the compress step: the global
            # output layout on every rank
            sizes = shard.gather_sizes(d_len, N_all)
            shard.global_offsets(sizes)

    for _ in range(args.warmup):
        step()
    D.barrier()
    eng.set_timing(True)
    phases = {}
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()  # back to back: the phase events are read after the timed region
    D.barrier()
    elapsed = D.max(time.perf_counter() - t0)
    for ph in PHASES_INFLATE:
        v = eng.last_ms(ph)  # summed over the timed steps
        if v >= 0:
            phases[ph] = phases.get(ph, 0.0) + v
    eng.set_timing(False)
    assert int((d_status != 1).sum()) == 0, "some members failed"
    out_local = int(d_len.to(torch.int64).sum())
    out_total = D.sum(out_local)
    in_local = len(blob)
    in_total = D.sum(in_local)
    # parity: every member's output against its source bytes / fixture digest (on the GPU), or,
    # where the reference's own decode differs from the source, against the reference's decode
    checked = bad = 0
    opts = dict(o.split("=", 1) for o in args.option)
    dname = GOLDENS_DEC.get((args.corpus, L, 6, enc_fmt)) if opts.get("inflate_ref_wrap", "1") != "0" else None
    if not args.no_verify:
        src = torch.frombuffer(host, dtype=torch.uint8).to(D.dev).view(-1, L)
        lens = d_len.cpu().tolist()
        drecs = None
        if dname:
            import golden_io
            drecs = golden_io.batch(dname)
        for i, e in enumerate(expect):
            if e[0] == "u" and drecs is not None:
                got = d_out[ooffs[i]:ooffs[i] + lens[i]].cpu().numpy().tobytes()
                ok = (lens[i], hashlib.sha256(got).digest()[:16]) == drecs[uniq[e[1]]]
            elif e[0] == "u":
                ok = lens[i] == L and bool(torch.equal(d_out[ooffs[i]:ooffs[i] + L], src[e[1]]))
            else:
                got = d_out[ooffs[i]:ooffs[i] + lens[i]].cpu().numpy().tobytes()
                ok = lens[i] == e[1] and hashlib.sha256(got).hexdigest() == e[2]
            checked += 1
            bad += not ok
        checked, bad = D.sum(checked), D.sum(bad)
        assert bad == 0, "%d of %d members decode wrong" % (bad, checked)
    extra = {}
    if D.world == 1 and D.rank == 0 and not args.no_shard_sweep:
        # what rank 0 decodes at 8 / 4 / 2 GPUs: the first shard_range(., G, 0) members of the same
        # global list (same device buffers, one GPU), each size timed over --steps back-to-back batches
        def step_n(m):
            eng.decompress_device(dec_fmt, m, d_in.data_ptr(), in_off, in_len, d_out.data_ptr(), out_off, out_cap,
                                  d_status.data_ptr(), d_phase.data_ptr(), d_msg.data_ptr(), d_len.data_ptr(),
                                  d_cons.data_ptr(), stream.cuda_stream)
        sweep = {}
        for g in (8, 4, 2):
            m = shard.shard_range(N, g, 0)[1]
            if m < 1 or m >= N:
                continue
            step_n(m)
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            for _ in range(args.steps):
                step_n(m)
            torch.cuda.synchronize()
            sweep[str(m)] = round((time.perf_counter() - t1) / args.steps * 1e3, 4)
            assert int((d_status[:m] != 1).sum()) == 0, "shard of %d members failed" % m
            if g == 8:  # the 8-GPU shard's phases (a separate pass: the timing events are not free)
                eng.set_timing(True)
                ph8 = {}
                for _ in range(args.steps):
                    step_n(m)
                    for ph in PHASES_INFLATE:
                        v = eng.last_ms(ph)
                        if v >= 0:
                            ph8[ph] = ph8.get(ph, 0.0) + v / args.steps
                eng.set_timing(False)
                extra["shard8_phase_ms"] = {k: round(v, 4) for k, v in ph8.items()}
        sweep[str(N)] = round(elapsed / args.steps * 1e3, 4)
        extra["shard_sweep_ms"] = sweep
        m8 = str(shard.shard_range(N, 8, 0)[1])
        if m8 in sweep:
            extra["implied_1_to_8_speedup"] = round(sweep[str(N)] / sweep[m8], 3)
    if D.world == 1 and D.rank == 0 and not args.no_e2e:
        # end-to-end: caller-owned host buffers -> host buffers through zs_inflate_batch
        import numpy as np
        hin = np.frombuffer(blob, dtype=np.uint8)
        hout = np.empty(oo, dtype=np.uint8)
        res = [(ctypes.c_int32 * N)() for _ in range(3)] + [(ctypes.c_uint32 * N)() for _ in range(2)]

        def e2e():
            eng.decompress_host(dec_fmt, N, hin.ctypes.data, in_off, in_len, hout.ctypes.data, out_off, out_cap, *res)
        e2e()
        t1 = time.perf_counter()
        reps = max(1, min(args.steps, 5))
        for _ in range(reps):
            e2e()
        te = (time.perf_counter() - t1) / reps
        ok = all(res[0][i] == 1 for i in range(N)) and sum(res[3]) == out_local
        extra["end_to_end"] = {"value": round(out_local / te / 1e6, 2), "unit": "MB/s (out)", "ms": round(te * 1e3, 3),
                               "path": "host buffers -> zs_inflate_batch (pinned staging, chunks whose copies "
                                       "overlap the kernels) -> host buffers", "matches_device_path": bool(ok)}
    if D.rank == 0:
        phase_avg = {k: round(v / args.steps, 4) for k, v in phases.items()}
        # the dominant KERNEL phase over the whole member list (inflate_join is the caller's stream waiting for
        # the side stream; the split decode and the fallback see a few members only -- C5-ii's fixtures --
        # and are not priced against the batch's bytes)
        side = ("inflate_join", "finish", "split_find", "split_decode", "split_resolve", "seg_find", "seg_fallback")
        dom = max((k for k in phase_avg if k not in side), key=phase_avg.get)
        k_ms = phase_avg[dom]
        alg = in_local + out_local  # compressed_in + uncompressed_out per member
        if dom in ("inflate_wave", "inflate_large"):  # only the members with more input than inflate_wave_min
            opts = dict(o.split("=", 1) for o in args.option)
            wmin = int(opts.get("inflate_wave_min", 32768))
            olen = d_len.cpu().tolist()
            alg = sum(len(m) + olen[i] for i, m in enumerate(members) if len(m) > wmin)
        achieved = alg / (k_ms / 1e3) / 1e9
        # the phase's kernel (profiles key template instances on their own: "zs_k_inflate_lane<true,true>")
        kernels = {"inflate_lane": ["zs_k_inflate_lane<0,false>", "zs_k_inflate_lane<1,false>",
                                    "zs_k_inflate_lane<2,false>"],
                   "inflate_large": ["zs_k_inflate_lane<2,true>", "zs_k_inflate_lane<0,true>"],
                   "inflate_wave": ["zs_k_inflate_wave<true>", "zs_k_inflate_wave<false>"]}.get(dom, ["zs_k_" + dom])
        traffic, tsrc = profiled_traffic(kernels, k_ms, profile_tag(args))
        ceil = profiled_ceilings(kernels, k_ms, profile_tag(args))
        kern = tsrc.split(" (")[1].split(" avg")[0] if traffic is not None else kernels[0]
        cpu = None
        if not (args.no_cpu_baseline or D.world > 1):
            import oracle
            key = {"deflate64-raw": "deflate64", "gzip": "gunzip"}.get(dec_fmt, "inflate")
            cpu = cpu_baseline(args, "member", lambda i: comp[i % len(comp)],
                               lambda m: oracle.decompress(m, dec_fmt, cap=L), L, N, key)
        name = {"deflate64-raw": "deflate64-raw decode (C5-ii)", "gzip": "gunzip + crc32 (C5-i)"}.get(
            dec_fmt, "inflate %s L6 members (C3)" % dec_fmt)
        if dec_fmt == "deflate-raw" and L == 262144:  # the C4 streams decoded back (reference-exact)
            name = "inflate deflate-raw L6, %d x 256 KiB members (C4 decoded back)" % N_glob
        line = {
            "metric": "uncompressed MB/s, %s" % name,
            "value": round(out_total / (elapsed / args.steps) / 1e6, 2), "unit": "MB/s", "n_gpus": D.world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "u8", "data": "synthetic",
            "config": {"workload": "%d members (%d unique %s-corpus %d B buffers x %d%s), %s decode" % (
                N_glob, S, args.corpus, L, R, " + the 9 reference deflate64 fixtures, sharded with them" if dec_fmt ==
                "deflate64-raw" else "", dec_fmt), "members_per_gpu": N, "compressed_bytes": in_total,
                "parallelism": "dp%d" % D.world},
            "verify": {"members_checked": checked, "mismatches": bad, "sources_vs_golden": members_checked,
                       "golden": "tests/golden/batch_%s.bin" % gname if gname else None,
                       "decode_golden": "tests/golden/batch_%s.bin" % dname if dname else None},
            "roofline": {"bound": "hbm", "kernel": kern, "achieved": round(achieved, 2),
                         "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 5),
                         "traffic": traffic, "traffic_source": tsrc, "algorithmic_bytes": alg,
                         "kernel_ms": round(k_ms, 4), "phase_ms": phase_avg,
                         "ceilings": ceil},
            "cpu_baseline": cpu,
        }
        line.update(extra)
        print(json.dumps(line), flush=True)
    D.close()


if __name__ == "__main__":
    main()
