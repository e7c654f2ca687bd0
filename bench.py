#!/usr/bin/env python3
"""Headline benchmark: uncompressed MB/s, deflate-raw level 6, 4096 x 64 KiB
synthetic T-corpus streams per GPU (BASELINE.json configs[1]).

One process per GPU (torch.distributed.run for N > 1).  A "step" is one batch
compression of the rank's 4096 streams, input already resident in HBM, output
written to HBM; rank r compresses stream indices [r*4096, (r+1)*4096) so the
per-GPU work is fixed (weak scaling).  For N > 1 the per-stream compressed
sizes are all-gathered over RCCL at the end of every step (the "final size
gather" of the north star: it gives every rank the global output layout).

Prints ONE JSON line on rank 0.  See DESIGN.md "Measurement".
"""
import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "zlib-streams-ts_amd"))

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s peak


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--streams", type=int, default=4096)
    ap.add_argument("--stream-bytes", type=int, default=65536)
    ap.add_argument("--level", type=int, default=6)
    ap.add_argument("--format", default="deflate-raw")
    ap.add_argument("--corpus", default="text")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="bounded CPU-baseline sample")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--verify", action="store_true", help="check every output against the batch golden")
    ap.add_argument("--mode", default="deflate", choices=["deflate", "inflate"],
                    help="deflate: the headline (configs[1]); inflate: C3 decode of pre-built members (configs[2])")
    ap.add_argument("--replicas", type=int, default=16, help="inflate: members = streams x replicas (C3: 4096 x 16)")
    return ap.parse_args()


def profiled_traffic(kernel):
    """HBM bytes per launch of `kernel` from the newest committed rocprofv3 PMC
    summary (FETCH_SIZE / WRITE_SIZE passes, gfx950 read correction applied by
    tools/summarize_profile.py), or (None, None)."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "*", "summary*.json")))
    for f in reversed(files):
        try:
            e = json.load(open(f)).get(kernel)
        except (OSError, ValueError):
            continue
        if e and "hbm_bytes_corrected" in e:
            return int(e["hbm_bytes_corrected"]), os.path.relpath(f, ROOT)
    return None, None


def cpu_baseline(args):
    """The C oracle (a single-threaded restatement of the reference algorithm),
    timed on a bounded sample of the same workload on this host."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle
    import zsamd

    oracle.lib()
    n = args.stream_bytes
    done, t_total, i = 0, 0.0, 0
    while t_total < args.cpu_seconds and i < args.streams:
        data = bytes(zsamd.corpus(args.corpus, i, 1, n, 1))
        t0 = time.perf_counter()
        st, out, _ = oracle.compress(data, args.level, args.format)
        t_total += time.perf_counter() - t0
        done += n
        i += 1
    return {"value": round(done / t_total / 1e6, 3), "unit": "MB/s", "cores": 1, "kind": "port",
            "sample": "%d of the %d x %d B %s streams, oracle/ C restatement, 1 thread" % (i, args.streams, n, args.corpus)}


def main():
    args = parse()
    if args.mode == "inflate":
        return main_inflate(args)
    import torch
    import torch.distributed as dist
    import zsamd

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    S, L = args.streams, args.stream_bytes
    first = rank * S
    host = zsamd.corpus(args.corpus, first, S, L, threads=8)
    d_in = torch.frombuffer(host, dtype=torch.uint8).to(dev)
    cap = zsamd.deflate_capacity(L, args.format)
    d_out = torch.zeros(S * cap, dtype=torch.uint8, device=dev)
    d_status = torch.zeros(S, dtype=torch.int32, device=dev)
    d_len = torch.zeros(S, dtype=torch.int32, device=dev)
    in_off = (ctypes.c_uint64 * S)(*[i * L for i in range(S)])
    in_len = (ctypes.c_uint32 * S)(*([L] * S))
    out_off = (ctypes.c_uint64 * S)(*[i * cap for i in range(S)])
    out_cap = (ctypes.c_uint32 * S)(*([cap] * S))
    eng = zsamd.Engine(local)
    stream = torch.cuda.current_stream(dev)
    import zsamd.shard as shard

    def step():
        eng.compress_device(args.level, args.format, S, d_in.data_ptr(), in_off, in_len, d_out.data_ptr(), out_off,
                            out_cap, d_status.data_ptr(), d_len.data_ptr(), stream.cuda_stream)
        if world > 1:
            # the final size gather (RCCL all_gather over xGMI): global output layout on every rank
            sizes = shard.gather_sizes(d_len, world * S)
            shard.global_offsets(sizes)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    eng.set_timing(True)
    phases = {}
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
        for ph in ("checksum", "prev", "depth", "match", "parse", "trees", "layout", "emit", "finish"):
            v = eng.last_ms(ph)
            if v >= 0:
                phases[ph] = phases.get(ph, 0.0) + v
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    eng.set_timing(False)
    t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())

    status = d_status.cpu()
    lens = d_len.cpu()
    assert int((status != 1).sum()) == 0, "some streams failed: %s" % status.unique()
    out_total = int(lens.sum())
    in_total = S * L
    if args.verify:
        import hashlib
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        import golden_io
        recs = golden_io.batch("t64_l6_raw")
        ob = d_out.cpu().numpy()
        for i in range(S):
            o = ob[i * cap: i * cap + int(lens[i])].tobytes()
            assert (len(o), hashlib.sha256(o).digest()[:16]) == recs[first + i], "stream %d differs" % (first + i)

    if rank == 0:
        ms_per_step = elapsed / args.steps * 1e3
        value = world * in_total / (elapsed / args.steps) / 1e6
        phase_avg = {k: round(v / args.steps, 4) for k, v in phases.items()}
        dom = max(phase_avg, key=phase_avg.get) if phase_avg else None
        roof = None
        if dom:
            alg = in_total + out_total  # bytes_in + bytes_out per stream, x streams per launch
            achieved = alg / (phase_avg[dom] / 1e3) / 1e9
            traffic, tsrc = profiled_traffic("zs_k_" + dom)
            roof = {"bound": "hbm", "kernel": dom, "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": traffic, "traffic_source": tsrc,
                    "algorithmic_bytes": alg, "kernel_ms": phase_avg[dom], "phase_ms": phase_avg,
                    "pipeline_ms": round(sum(phase_avg.values()), 4)}
        cpu = None if (args.no_cpu_baseline or world > 1) else cpu_baseline(args)
        line = {
            "metric": "uncompressed MB/s, deflate-raw L6, 4096x64KiB batch at 1/2/4/8 GPUs",
            "value": round(value, 2), "unit": "MB/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4), "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": "u8", "data": "synthetic",
            "config": {"workload": "%d x %d B %s-corpus streams per GPU, %s level %d" % (S, L, args.corpus, args.format,
                                                                                          args.level),
                       "streams_per_gpu": S, "stream_bytes": L, "level": args.level, "format": args.format,
                       "compressed_bytes_per_gpu": out_total, "ratio": round(in_total / max(1, out_total), 4),
                       "parallelism": "dp%d" % world},
            "roofline": roof, "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


def main_inflate(args):
    """C3: 4096 unique M-corpus 64 KiB buffers compressed at
    deflate-raw L6 (by this engine, bit-exact to the reference; the batch golden
    is checked), replicated x16 = 65,536 members, decoded on one GPU.  Metric:
    uncompressed (output) MB/s.  Weak scaling: rank r decodes its own copy."""
    import torch
    import torch.distributed as dist
    import zsamd

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    S, L, R = args.streams, args.stream_bytes, args.replicas
    eng = zsamd.Engine(local)
    host = zsamd.corpus("mixed", 0, S, L, threads=8)
    comp = eng.compress_batch([bytes(host[i * L:(i + 1) * L]) for i in range(S)], "deflate-raw", 6)
    members = comp * R
    N = len(members)
    blob = b"".join(members)
    d_in = torch.frombuffer(bytearray(blob), dtype=torch.uint8).to(dev)
    offs, o = [], 0
    for m in members:
        offs.append(o)
        o += len(m)
    in_off = (ctypes.c_uint64 * N)(*offs)
    in_len = (ctypes.c_uint32 * N)(*[len(m) for m in members])
    cap = L
    d_out = torch.zeros(N * cap, dtype=torch.uint8, device=dev)
    out_off = (ctypes.c_uint64 * N)(*[i * cap for i in range(N)])
    out_cap = (ctypes.c_uint32 * N)(*([cap] * N))
    i32 = lambda: torch.zeros(N, dtype=torch.int32, device=dev)
    d_status, d_phase, d_msg, d_len, d_cons = i32(), i32(), i32(), i32(), i32()
    stream = torch.cuda.current_stream(dev)

    def step():
        eng.decompress_device("deflate-raw", N, d_in.data_ptr(), in_off, in_len, d_out.data_ptr(), out_off, out_cap,
                              d_status.data_ptr(), d_phase.data_ptr(), d_msg.data_ptr(), d_len.data_ptr(),
                              d_cons.data_ptr(), stream.cuda_stream)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    eng.set_timing(True)
    phases = {}
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
        for ph in ("inflate_lane", "inflate_check", "inflate", "finish"):
            v = eng.last_ms(ph)
            if v >= 0:
                phases[ph] = phases.get(ph, 0.0) + v
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    eng.set_timing(False)
    t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())
    assert int((d_status != 1).sum()) == 0, "some members failed"
    assert int(d_len.sum()) == N * L
    if args.verify:
        ob = d_out.cpu().numpy()
        for i in range(S):
            assert ob[i * cap:(i + 1) * cap].tobytes() == bytes(host[i * L:(i + 1) * L]), "member %d differs" % i
    if rank == 0:
        out_total, in_total = N * L, len(blob)
        phase_avg = {k: round(v / args.steps, 4) for k, v in phases.items()}
        dom = max(phase_avg, key=phase_avg.get)
        k_ms = phase_avg[dom]
        alg = in_total + out_total  # compressed_in + uncompressed_out per member
        achieved = alg / (k_ms / 1e3) / 1e9
        cpu = None
        if not (args.no_cpu_baseline or world > 1):
            sys.path.insert(0, os.path.join(ROOT, "tests"))
            import oracle
            done, tt, i = 0, 0.0, 0
            while tt < args.cpu_seconds and i < S:
                t1 = time.perf_counter()
                oracle.decompress(comp[i], "deflate-raw", cap=L)
                tt += time.perf_counter() - t1
                done += L
                i += 1
            cpu = {"value": round(done / tt / 1e6, 3), "unit": "MB/s", "cores": 1, "kind": "port",
                   "sample": "%d of the %d unique members, oracle/ C restatement, 1 thread" % (i, S)}
        line = {
            "metric": "uncompressed MB/s, inflate deflate-raw L6 members (C3)",
            "value": round(world * out_total / (elapsed / args.steps) / 1e6, 2), "unit": "MB/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u8", "data": "synthetic",
            "config": {"workload": "%d members (%d unique M-corpus %d B buffers x %d), deflate-raw L6, decode" % (N, S, L, R),
                       "members_per_gpu": N, "compressed_bytes_per_gpu": in_total, "parallelism": "dp%d" % world},
            "roofline": {"bound": "hbm", "kernel": dom, "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 5),
                         "traffic": profiled_traffic("zs_k_" + dom)[0], "traffic_source": profiled_traffic("zs_k_" + dom)[1],
                         "algorithmic_bytes": alg, "kernel_ms": round(k_ms, 4), "phase_ms": phase_avg},
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
