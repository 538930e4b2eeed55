#!/usr/bin/env python3
"""bench.py — rows/s and HBM roofline of the 1B-row int32 select+sum (BASELINE.json).

A step is one pass of the hot path over one batch: range select [N/4, N/4 + N/100)
(1 % selectivity) + count + exact int64 sum over a 1e9-row int32 column that is
already resident in HBM (libmq mq_select_agg: k_scan + k_final). N=1 is
BASELINE configs[1]; with --gpus G each rank scans its own 1e9-row column
(seeds 42..42+G-1, configs[3]) and the per-rank {count, sum} are combined by one
RCCL all-reduce inside the step ("weak" scaling); the all-reduce runs on its own
stream, overlapped with the next step's scan (double-buffered aggregates). Data are synthetic
(SURVEY.md §8(c) generator), generated on the device.

  python bench.py [--gpus N --steps K --warmup W] [--rows R] [--no-cpu] [--no-extra]
  python bench.py --inproc [--gpus N]   libmq's own row-shard path, one process (inproc_main)

Rank 0 prints ONE JSON line. Roofline: algorithmic bytes 4N per scan launch ÷ the
scan kernel's mean duration from HIP events on the launch stream. cpu_baseline:
the reference's own query.c (oracle/_ref/libref.so) select_column -> fetch_column
-> sum on a bounded sample, single thread, on this box's host.
"""
from __future__ import annotations

import argparse
import ctypes as C
import importlib.util
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "analytical-database_amd")
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)


def _load(name, path):
    if name not in sys.modules:
        spec = importlib.util.spec_from_file_location(name, path)
        mod = importlib.util.module_from_spec(spec)
        sys.modules[name] = mod
        spec.loader.exec_module(mod)
    return sys.modules[name]


def cpu_baseline(rows: int) -> dict:
    """Reference CPU path on a bounded sample of the same workload (rank 0, N=1)."""
    import numpy as np
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import refcpu  # checker / baseline only
    from refapi import Api, make_column

    ns = min(rows, 250_000_000)
    lo, hi = int(0.25 * ns), int(0.25 * ns) + int(0.01 * ns)
    d = refcpu.gen_uniform(ns, 42, nthreads=16)
    kind = "reference" if refcpu.have_reference() else "port"
    times = []
    if kind == "reference":
        api = Api(refcpu.reference())
        col = make_column(d)
        for _ in range(3):
            t0 = time.perf_counter()
            pos = api.select_column(col, lo, hi)
            vals = api.fetch_column(col, pos)
            s = api.sum_result(vals)
            times.append(time.perf_counter() - t0)
    else:
        for _ in range(3):
            t0 = time.perf_counter()
            pos = refcpu.select_scan(d, lo, hi)
            s = refcpu.agg(refcpu.fetch(d, pos))["sum"]
            times.append(time.perf_counter() - t0)
    t1 = statistics.median(times)
    # host-cores variant: row-balanced pthreads restatement on every core this
    # process may use (SURVEY §8(d) "nproc threads"; on the GPU box the cgroup CPU
    # quota, not nproc, is the limit, and the record says which)
    cores, why = host_cores()
    mt = []
    for _ in range(3):
        t0 = time.perf_counter()
        c, s2 = refcpu.count_sum(d, lo, hi, nthreads=cores)
        mt.append(time.perf_counter() - t0)
    assert s2 == s
    variants = {"host_cores": {"value": ns / statistics.median(mt), "cores": cores, "kind": "port",
                               "cores_from": why,
                               "what": f"refcpu rc_select_count_sum, {cores} pthreads, row-balanced"}}
    if kind == "reference":
        # the reference as its Makefile builds it (-O0, src/Makefile:12), one run
        api0 = Api(refcpu.reference(refcpu.REFLIB_O0))
        t0 = time.perf_counter()
        s0 = api0.sum_result(api0.fetch_column(col, api0.select_column(col, lo, hi)))
        variants["reference_O0"] = {"value": ns / (time.perf_counter() - t0), "cores": 1,
                                    "kind": "reference", "what": "same chain, libref_O0.so"}
        assert s0 == s
        # the reference's own 3-thread shared_select (query.c:496-583), one query
        t0 = time.perf_counter()
        api.shared_select(col, [lo], [hi])
        variants["shared_select_3threads"] = {"value": ns / (time.perf_counter() - t0), "cores": 3,
                                              "kind": "reference",
                                              "what": "shared_select Q=1, value-range split"}
    return {"value": ns / t1, "unit": "rows/s", "cores": 1, "kind": kind,
            "sample": f"{ns} rows int32 uniform [0,{ns}) seed 42, select [{lo},{hi}) -> "
                      f"fetch -> sum, {'oracle/_ref/libref.so (reference query.c, gcc -O2)' if kind == 'reference' else 'oracle/refcpu.c -O2'}, "
                      f"median of 3 = {t1:.3f} s",
            "variants": variants,
            "nproc": os.cpu_count(), "cpu_model": _cpu_model()}


def host_cores() -> tuple[int, str]:
    """Cores this process may run on: min(affinity mask, cgroup v2 cpu.max quota)."""
    n = len(os.sched_getaffinity(0))
    why = f"sched_getaffinity={n} (nproc={os.cpu_count()})"
    try:
        quota, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if quota != "max":
            q = max(1, int(int(quota) // int(period)))
            why += f", cgroup cpu.max quota={q}"
            n = min(n, q)
    except (OSError, ValueError):
        pass
    return n, why


def _cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def launch_ranks(ngpus: int, argv: list) -> int:
    """`bench.py --gpus N` without an external launcher: start N rank processes of
    this script (one per GPU, RANK/LOCAL_RANK/WORLD_SIZE/MASTER_* set as
    torch.distributed.run sets them) before this process touches the GPU, wait for
    all, return the worst exit status. Rank 0 prints the JSON line."""
    import socket
    import subprocess
    if os.environ.get("MQ_BENCH_ONE_DEVICE") != "1":
        import torch  # device_count() does not initialise the GPU on this image
        have = torch.cuda.device_count()
        if ngpus > have:
            print(f"bench.py: --gpus {ngpus} but only {have} GPU(s) visible", file=sys.stderr)
            return 2
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = []
    for r in range(ngpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(ngpus),
                   LOCAL_WORLD_SIZE=str(ngpus), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + argv, env=env))
    codes = [p.wait() for p in procs]
    bad = [c for c in codes if c != 0]
    return bad[0] if bad else 0


def inproc_main(args) -> None:
    """--inproc: libmq's own multi-GPU path (mq_shard.c) in ONE process, as the
    reference server would run it after linking libmq: one 1e9-row column (a memfd
    file mapping, like the reference's column files) split into --gpus row shards,
    shard g resident on GPU g (mq_shard_config) with a host thread and stream of its
    own; a step is the reference's chain select_column -> fetch_column -> sum
    (server.c:137-247), each operator running on every shard and concatenating /
    folding in shard order. PCIe-inclusive (the API returns host payloads), total
    work fixed ("strong"). MQ_BENCH_ONE_DEVICE=1 puts every shard on GPU 0 (a
    rehearsal of the split on a one-GPU box). Parity: K and the sum against the
    reference's goldens (seed 42)."""
    import mmap
    import numpy as np
    import torch
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    mq = _load("mq_binding", os.path.join(PKG, "mq.py"))
    from refapi import make_column, _libc
    ng = args.gpus
    devices = [0] * ng if os.environ.get("MQ_BENCH_ONE_DEVICE") == "1" else list(range(ng))
    lib = mq.load()
    mq.check(lib.mq_init(0), "mq_init")
    n = args.rows
    lo = int(0.25 * n)
    hi = lo + int(args.sel * n)
    # the §8(c) column, generated on the device and copied into a file mapping
    fd = os.memfd_create("col")
    os.ftruncate(fd, 4 * n)
    m = mmap.mmap(fd, 4 * n, mmap.MAP_SHARED, mmap.PROT_READ | mmap.PROT_WRITE)
    os.close(fd)
    host = np.frombuffer(m, dtype=np.int32)
    g = torch.empty(n, dtype=torch.int32, device="cuda")
    mq.check(lib.mq_gen_uniform(g.data_ptr(), n, 42, n, None), "gen")
    torch.cuda.synchronize()
    host[:] = g.cpu().numpy()
    del g
    torch.cuda.empty_cache()
    col = make_column(host, b"col")
    arr = (C.c_int * ng)(*devices)
    mq.check(lib.mq_shard_config(ng, arr, ng, 0), "mq_shard_config")
    t0 = time.perf_counter()
    mq.check(lib.mq_column_upload(C.byref(col)), "upload")
    t_up = time.perf_counter() - t0
    lo_c, hi_c = C.c_int(lo), C.c_int(hi)
    step_s, k, total = [], None, None
    for i in range(args.warmup + args.steps):
        st = mq.Status(0, None)
        t0 = time.perf_counter()
        rp = lib.select_column(C.byref(col), C.byref(lo_c), C.byref(hi_c), C.byref(st))
        rf = lib.fetch_column(C.byref(col), rp, C.byref(st)) if st.code == mq.OK else None
        gc = mq.GeneralizedColumn()
        gc.column_type = mq.RESULT
        gc.column_pointer.result = rf
        rs = lib.sum(C.byref(gc), C.byref(st)) if st.code == mq.OK else None
        dt = time.perf_counter() - t0
        if st.code != mq.OK:
            print(f"bench.py --inproc: operator failed: {st.error_message}", file=sys.stderr)
            sys.exit(1)
        k = rp.contents.num_tuples
        total = C.cast(rs.contents.payload, C.POINTER(C.c_longlong))[0]
        for r in (rp, rf, rs):
            _libc.free(r.contents.payload)
            _libc.free(r)
        if i >= args.warmup:
            step_s.append(dt)
    resid = mq.residency(lib)
    lib.mq_release_all()
    gold = json.load(open(os.path.join(ROOT, "tests", "golden", "goldens.json")))
    join = None if args.no_join else inproc_join_leg(lib, mq, torch, devices, gold)
    mq.check(lib.mq_shard_config(0, None, 0, 0), "mq_shard_config reset")
    want = next((r for r in gold["config4"] if r["n"] == n and r["seed"] == 42 and r["low"] == lo and r["high"] == hi),
                None)
    parity = None if want is None else (k, total) == (want["k"], want["sum"])
    elapsed = sum(step_s)
    out = {
        "metric": "rows/sec, 1B-row int32 select -> fetch -> sum through libmq's drop-in API "
                  "(PCIe-inclusive), one process, row shards over N GPUs",
        "value": n * len(step_s) / elapsed,
        "unit": "rows/s",
        "n_gpus": ng,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": 1e3 * elapsed / len(step_s),
        "ms_per_step_median": 1e3 * statistics.median(step_s),
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "int32",
        "data": "synthetic",
        "config": {"workload": "select_column -> fetch_column -> sum on one 1e9-row column, row-sharded",
                   "rows": n, "selectivity": args.sel, "low": lo, "high": hi, "shards": ng,
                   "devices": devices, "parallelism": f"row shards x{ng} (mq_shard.c), one process"},
        "ms_upload": 1e3 * t_up,
        "upload_gbs": 4.0 * n / t_up / 1e9,
        "residency": resid,
        "parity": {"ok": parity, "count": k, "sum": total},
        "extra": {"config5_partitioned_join": join},
    }
    bad = parity_failures(out)
    out["parity_failures"] = bad
    print(json.dumps(out), flush=True)
    if parity is False or bad:
        print("bench.py --inproc: parity FAILED", file=sys.stderr)
        sys.exit(1)


def inproc_join_leg(lib, mq, torch, devices, gold, logn: int = 28, reps: int = 3) -> dict:
    """Config 5 (2^28 x 2^28 hash join, SURVEY §8(c) keys) key-partitioned over the row
    shards (mq_shard_join): each side split into len(devices) contiguous
    row ranges, range g resident on devices[g]; partition, exchange (peer copies), local
    joins, return exchange, place. Device-resident inputs and outputs (no PCIe). Parity:
    M and the FNV-1a of the concatenated pairs against the reference's goldens."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import refcpu  # checker only (pair hash)
    G = len(devices)
    n = 1 << logn
    full = [torch.empty(n, dtype=torch.int32, device="cuda:0") for _ in range(3)]
    mq.check(lib.mq_gen_join_keys(full[0].data_ptr(), n, 0, None))
    mq.check(lib.mq_gen_join_keys(full[1].data_ptr(), n, 1, None))
    mq.check(lib.mq_gen_iota(full[2].data_ptr(), n, None))
    torch.cuda.synchronize()
    b = [n * g // G for g in range(G + 1)]
    pieces = [[x[b[g]:b[g + 1]].to(f"cuda:{devices[g]}") for x in full] for g in range(G)]
    del full
    torch.cuda.synchronize()
    V, U = C.c_void_p * G, C.c_uint64 * G
    c1 = V(*[pieces[g][0].data_ptr() for g in range(G)])
    c2 = V(*[pieces[g][1].data_ptr() for g in range(G)])
    pp = V(*[pieces[g][2].data_ptr() for g in range(G)])
    ns = U(*[b[g + 1] - b[g] for g in range(G)])
    times, phases = [], []
    o1 = o2 = m = None
    for rep in range(reps + 1):
        if o1 is not None:
            for g in range(G):
                lib.mq_pool_free(o1[g])
                lib.mq_pool_free(o2[g])
        o1, o2, m = V(), V(), U()
        t0 = time.perf_counter()
        mq.check(lib.mq_shard_join(c1, pp, ns, c2, pp, ns, o1, o2, m), "mq_shard_join")
        dt = time.perf_counter() - t0
        ph = (C.c_double * 4)()
        lib.mq_shard_join_times(ph)
        if rep:
            times.append(dt)
            phases.append(list(ph))
    import numpy as np
    parts = []
    for g in range(G):
        a1, a2 = np.empty(m[g], np.int32), np.empty(m[g], np.int32)
        for a, o in ((a1, o1), (a2, o2)):
            if m[g]:
                mq.check(lib.mq_memcpy_d2h(a.ctypes.data, o[g], a.nbytes, None))
        parts.append((a1, a2))
        lib.mq_pool_free(o1[g])
        lib.mq_pool_free(o2[g])
    M = int(sum(m))
    fnv = refcpu.fnv1a64_pairs(np.concatenate([p[0] for p in parts]), np.concatenate([p[1] for p in parts]))
    want = [r for r in gold["join_survey"] if r["n"] == n]
    ok = bool(want) and (M, f"{fnv:016x}") == (want[0]["m"], want[0]["pairs_fnv1a64"])
    del pieces
    t = statistics.median(times)
    k = len(times) // 2
    return {"n_build": n, "n_probe": n, "m": M, "shards": G, "devices": devices, "ms": 1e3 * t,
            "rows_per_s": 2 * n / t, "algorithmic_bytes": 16 * n + 8 * M,
            "ms_phases": dict(zip(("partition", "exchange_join", "return_place", "total"),
                                  sorted(phases, key=lambda x: x[3])[k])),
            "pairs_per_shard": list(m), "parity": ok,
            "note": "mq_shard_join wall time (host), device-resident inputs and outputs; on one GPU "
                    "(MQ_BENCH_ONE_DEVICE=1) every shard and exchange shares device 0"}


def main() -> None:
    if "--api-child" in sys.argv[1:]:
        ap = argparse.ArgumentParser()
        ap.add_argument("--api-child", action="store_true")
        ap.add_argument("--rows", type=int, default=1_000_000_000)
        ap.add_argument("--lo", type=int, required=True)
        ap.add_argument("--hi", type=int, required=True)
        api_child(ap.parse_args())
        return
    if "--inproc" in sys.argv[1:]:
        ap = argparse.ArgumentParser()
        ap.add_argument("--inproc", action="store_true")
        ap.add_argument("--gpus", type=int, default=1)
        ap.add_argument("--steps", type=int, default=10)
        ap.add_argument("--warmup", type=int, default=2)
        ap.add_argument("--rows", type=int, default=1_000_000_000)
        ap.add_argument("--sel", type=float, default=0.01)
        ap.add_argument("--no-join", action="store_true", help="skip the partitioned-join leg")
        inproc_main(ap.parse_args())
        return
    if "WORLD_SIZE" not in os.environ:
        pre = argparse.ArgumentParser(add_help=False)
        pre.add_argument("--gpus", type=int, default=1)
        known, _ = pre.parse_known_args()
        if known.gpus > 1:
            sys.exit(launch_ranks(known.gpus, sys.argv[1:]))
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--rows", type=int, default=1_000_000_000)
    ap.add_argument("--sel", type=float, default=0.01)
    ap.add_argument("--no-cpu", action="store_true", help="skip the cpu_baseline leg")
    ap.add_argument("--no-extra", action="store_true", help="skip the positions/config-3 legs")
    ap.add_argument("--join", action="store_true",
                    help="N > 1: also time config 5 key-partitioned over the ranks (dist.partitioned_join)")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    mq = _load("mq_binding", os.path.join(PKG, "mq.py"))
    mqd = _load("mq_dist", os.path.join(PKG, "dist.py"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr)
        sys.exit(2)
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # Rehearsal knobs for the N > 1 path on a one-GPU box (never set by the driver):
    # MQ_BENCH_BACKEND=gloo and MQ_BENCH_ONE_DEVICE=1 put every rank on GPU 0
    # (RCCL refuses two ranks per GPU; gloo combines through host memory).
    if os.environ.get("MQ_BENCH_ONE_DEVICE") == "1":
        local = 0
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        backend = os.environ.get("MQ_BENCH_BACKEND", "nccl")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)

    lib = mq.load()
    mq.check(lib.mq_init(local), "mq_init")
    stream = torch.cuda.Stream(device=dev)
    sp = mq.stream_of(stream)
    n = args.rows
    seed = 42 + rank
    lo = int(0.25 * n)
    hi = lo + int(args.sel * n)

    with torch.cuda.stream(stream):
        col = torch.empty(n, dtype=torch.int32, device=dev)
        ws_bytes = lib.mq_scan_workspace_bytes(n)
        ws = torch.empty(ws_bytes, dtype=torch.uint8, device=dev)
        # two aggregate buffers: step i scans into aggs[i % 2] on `stream` while the
        # RCCL all-reduce of step i-1 runs on `comm`, so the combine (N > 1) is off
        # the scan's critical path; a buffer is rescanned only after its all-reduce
        aggs = [mqd.agg_tensor(dev), mqd.agg_tensor(dev)]
        comm = torch.cuda.Stream(device=dev)
        pending = [None, None]
        counter = [0]
        mq.check(lib.mq_gen_uniform(col.data_ptr(), n, seed, n, sp), "gen")

        def step(ev0=None, ev1=None):
            b = counter[0] % 2
            counter[0] += 1
            agg = aggs[b]
            if pending[b] is not None:
                stream.wait_event(pending[b])
            # one launch: k_scan<kSum> with the partials folded by the last block
            if ev0 is not None:
                ev0.record(stream)
            mq.check(lib.mq_select_sum(col.data_ptr(), n, 1, lo, 1, hi, agg.data_ptr(),
                                       ws.data_ptr(), ws_bytes, sp), "select_sum")
            if ev1 is not None:
                ev1.record(stream)
            if world > 1:
                scanned = torch.cuda.Event()
                scanned.record(stream)
                comm.wait_event(scanned)
                with torch.cuda.stream(comm):
                    mqd.combine_count_sum(agg)
                    fin = torch.cuda.Event()
                    fin.record(comm)
                pending[b] = fin

        for _ in range(args.warmup):
            step()
        evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
               for _ in range(args.steps)]
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(args.steps):
            step(*evs[i])
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        elapsed = time.perf_counter() - t0
        agg = aggs[(counter[0] - 1) % 2]  # the last step's combined aggregate
        kernel_ms = [a.elapsed_time(b) for a, b in evs]

    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        km = torch.tensor([statistics.mean(kernel_ms)], dtype=torch.float64, device=dev)
        dist.all_reduce(km, op=dist.ReduceOp.MAX)
        k_mean_ms = float(km.item())
    else:
        k_mean_ms = statistics.mean(kernel_ms)

    # parity of the last step against the reference goldens (tests/golden/goldens.json)
    res = mqd.unpack(agg)
    gold = json.load(open(os.path.join(ROOT, "tests", "golden", "goldens.json")))
    parity = None
    if n == 1_000_000_000 and abs(args.sel - 0.01) < 1e-12:
        rows = {r["seed"]: r for r in gold["config4"]}
        want_k = sum(rows[s]["k"] for s in range(42, 42 + world))
        want_s = sum(rows[s]["sum"] for s in range(42, 42 + world))
        parity = (res["count"], res["sum"]) == (want_k, want_s)

    achievable = achievable_read_peak(lib, mq, torch, stream, col, ws) if world == 1 else None

    extra = {}
    if world > 1 and args.join:  # every rank takes part (all_to_all exchanges)
        extra["config5_partitioned_join"] = dist_join_leg(lib, mq, mqd, torch, dist, dev, rank, world, gold)
    if rank == 0 and world == 1 and not args.no_extra:
        extra = extra_legs(lib, mq, torch, dev, stream, col, ws, ws_bytes, n, lo, hi, gold,
                           cpu=not args.no_cpu)

    bad = []
    if rank == 0:
        ms_step = 1e3 * elapsed / args.steps
        gbs = 4.0 * n / (k_mean_ms * 1e-3) / 1e9
        traffic = traffic_per_launch(n)
        out = {
            "metric": "rows/sec scanned + HBM GB/s (% of roofline), 1B-row int32 select+sum",
            "value": world * n * args.steps / elapsed,
            "unit": "rows/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_step,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "int32",
            "data": "synthetic",
            "config": {"workload": ("1B-row single int32 column, range select + sum"
                                    if world == 1 else
                                    f"{world}x independent 1B-row select+sum, one per GPU, "
                                    "RCCL all-reduce of {count,sum}"),
                       "rows_per_gpu": n, "selectivity": args.sel, "low": lo, "high": hi,
                       "parallelism": f"shard-by-query x{world}" if world > 1 else "single GPU"},
            "hbm_gbs_step": 4.0 * n * world / (elapsed / args.steps) / 1e9 / world,
            "roofline": {"bound": "hbm", "kernel": "k_scan<kSum,true> (mq_select_sum: count+sum, partials folded in-kernel)",
                         "achieved": gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": gbs / HBM_PEAK_GBS, "traffic": traffic[0], "traffic_source": traffic[1],
                         "kernel_ms_mean": k_mean_ms, "kernel_ms_min": min(kernel_ms),
                         "kernel_ms_median": statistics.median(kernel_ms),
                         "stream_read_probe": achievable,
                         "algorithmic_bytes_per_launch": 4 * n},
            "parity": {"ok": parity, "count": res["count"], "sum": res["sum"]},
            "extra": extra,
        }
        if world == 1 and not args.no_cpu:
            out["cpu_baseline"] = cpu_baseline(n)
        bad = parity_failures(out)
        out["parity_failures"] = bad
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()
    # fail loudly: a wrong combined count/sum on any rank, or any
    # extra leg's parity check false on rank 0, makes the run exit non-zero after the
    # JSON line is out
    if parity is False or (rank == 0 and bad):
        print(f"bench.py: parity FAILED: {'headline' if parity is False else ''} {bad}", file=sys.stderr)
        sys.exit(1)


def dist_join_leg(lib, mq, mqd, torch, dist, dev, rank, world, gold, logn: int = 28, reps: int = 3) -> dict:
    """Config 5 (2^28 x 2^28, SURVEY §8(c) keys) key-partitioned over the ranks, one per
    GPU (dist.partitioned_join: libmq's partition / local join / place kernels, RCCL
    all_to_all exchanges): rank r holds rows [r n / N, (r + 1) n / N) of both sides. Time =
    max over ranks, between barriers. Parity: the total M equals the reference's golden,
    and every rank's pairs join equal keys in probe-major, build-ascending order (with
    the identity positions and unique build keys this fixes the output)."""
    n = 1 << logn
    a, b = n * rank // world, n * (rank + 1) // world
    c1 = torch.empty(b - a, dtype=torch.int32, device=dev)
    c2 = torch.empty(b - a, dtype=torch.int32, device=dev)
    full = torch.empty(n, dtype=torch.int32, device=dev)
    mq.check(lib.mq_gen_join_keys(full.data_ptr(), n, 0, None))
    c1.copy_(full[a:b])
    mq.check(lib.mq_gen_join_keys(full.data_ptr(), n, 1, None))
    c2.copy_(full[a:b])
    p = torch.arange(a, b, dtype=torch.int32, device=dev)
    ph = mqd.LibmqPhases(lib, mq)
    ts = []
    for rep in range(reps + 1):
        torch.cuda.synchronize()
        dist.barrier()
        t0 = time.perf_counter()
        o1, o2 = mqd.partitioned_join(ph, c1, p, c2, p)
        torch.cuda.synchronize()
        dist.barrier()
        t = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        if rep:
            ts.append(float(t.item()))
    mq.check(lib.mq_gen_join_keys(full.data_ptr(), n, 0, None))
    bk = full[o1.long()] if o1.numel() else o1
    mq.check(lib.mq_gen_join_keys(full.data_ptr(), n, 1, None))
    pk = full[o2.long()] if o2.numel() else o2
    ok = bool(torch.equal(bk, pk))
    if o2.numel() > 1:
        ok = ok and bool((o2[1:] > o2[:-1]).all()) and int(o2[0]) >= a and int(o2[-1]) < b
    m = torch.tensor([o1.numel(), int(ok)], dtype=torch.int64, device=dev)
    dist.all_reduce(m, op=dist.ReduceOp.SUM)
    want = [r for r in gold["join_survey"] if r["n"] == n]
    t = statistics.median(ts)
    return {"n_build": n, "n_probe": n, "m": int(m[0]), "ranks": world, "ms": 1e3 * t, "rows_per_s": 2 * n / t,
            "parity": bool(want) and int(m[0]) == want[0]["m"] and int(m[1]) == world,
            "note": "strong scaling of config 5: the 2^28 x 2^28 join split over the ranks, exchanges by RCCL "
                    "all_to_all (DESIGN.md §6)"}


def parity_failures(out: dict) -> list:
    """Paths of every parity flag in the record that is False (headline and extras)."""
    bad = []

    def walk(x, path):
        if isinstance(x, dict):
            for k, v in x.items():
                p = f"{path}/{k}"
                if (k.startswith("parity") or k in ("ok", "identical")) and v is False:
                    bad.append(p)
                walk(v, p)

    walk(out, "")
    return bad


def achievable_read_peak(lib, mq, torch, stream, col, ws, launches: int = 20) -> dict:
    """SURVEY §8(d) 'achievable peak': k_stream_read (k_scan's loads, no predicate)
    over the same resident column, HIP events on the launch stream, median of
    `launches` after 3 warm-ups."""
    sp = mq.stream_of(stream)
    nbytes = C.c_uint64()
    ms = []
    with torch.cuda.stream(stream):
        for i in range(3 + launches):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(stream)
            mq.check(lib.mq_stream_read(col.data_ptr(), col.numel(), ws.data_ptr(), ws.numel(),
                                        C.byref(nbytes), sp), "stream_read")
            b.record(stream)
            b.synchronize()
            if i >= 3:
                ms.append(a.elapsed_time(b))
    med = statistics.median(ms)
    return {"kernel": "k_stream_read", "gbs": nbytes.value / (med * 1e-3) / 1e9,
            "bytes": nbytes.value, "ms_median": med}


def pcie_probe(torch, dev, stream, nbytes: int = 256 << 20, reps: int = 5) -> dict:
    """The host link's rate on this box: hipMemcpy of a 256 MB
    pinned host buffer to and from HBM (torch pinned tensors, copies on `stream`),
    median of `reps` after one warm-up. The drop-in API's transfers (api_leg) are
    judged against these."""
    h = torch.empty(nbytes, dtype=torch.uint8).pin_memory()
    d = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    out = {"bytes": nbytes}
    with torch.cuda.stream(stream):
        for name, fn in (("h2d", lambda: d.copy_(h, non_blocking=True)),
                         ("d2h", lambda: h.copy_(d, non_blocking=True))):
            ts = []
            for i in range(reps + 1):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                fn()
                torch.cuda.synchronize()
                if i:
                    ts.append(time.perf_counter() - t0)
            out[f"{name}_gbs"] = nbytes / statistics.median(ts) / 1e9
    del h, d
    return out


def print_leg(lib, mq, torch, dev, stream, pos, k, cpu: bool = True) -> dict:
    """print (query.c:245-304) of config 2's K positions: GPU formatting
    (mq_format_int32 + D2H of the text) vs the reference's sprintf loop on the
    same values (oracle/_ref/libref.so, host)."""
    import numpy as np
    sp = mq.stream_of(stream)
    out_d = torch.empty(12 * k, dtype=torch.uint8, device=dev)
    ws = torch.empty(lib.mq_format_workspace_bytes(k), dtype=torch.uint8, device=dev)
    host = torch.empty(12 * k, dtype=torch.uint8).pin_memory()
    ln = C.c_uint64()
    ms = []
    with torch.cuda.stream(stream):
        for i in range(4):
            t0 = time.perf_counter()
            mq.check(lib.mq_format_int32(pos.data_ptr(), k, out_d.data_ptr(), C.byref(ln),
                                         ws.data_ptr(), ws.numel(), sp))
            mq.check(lib.mq_memcpy_d2h(host.data_ptr(), out_d.data_ptr(), ln.value, sp))
            mq.check(lib.mq_stream_sync(sp))
            if i:
                ms.append(1e3 * (time.perf_counter() - t0))
    res = {"k": k, "bytes": ln.value, "ms_gpu_incl_d2h": statistics.median(ms)}
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import refcpu  # baseline only
    if cpu and refcpu.have_reference():
        from refapi import Api
        vals = pos[:k].cpu().numpy()
        api = Api(refcpu.reference())
        t0 = time.perf_counter()
        s_ref = api.print([(vals, mq.INT)])
        res["ms_cpu_reference"] = 1e3 * (time.perf_counter() - t0)
        res["identical"] = s_ref.encode() == host[:ln.value].numpy().tobytes()
    return res


def traffic_per_launch(n: int):
    """(HBM bytes per k_scan launch, source) from the newest round's committed rocprofv3
    PMC summary with a k_scan row for this N (profiles/rNN_pmc_traffic.json, written by
    tools/pmc_traffic.py from separate --pmc FETCH_SIZE / WRITE_SIZE passes: FETCH_SIZE
    x 2 for gfx950's halving, MI355X_MICROARCH.md §HBM, + WRITE_SIZE). (None, None) when
    no round has one."""
    import glob
    import re
    found = []
    for path in glob.glob(os.path.join(ROOT, "profiles", "r[0-9][0-9]_pmc_traffic*.json")):
        mr = re.match(r"r(\d\d)_", os.path.basename(path))
        try:
            row = json.load(open(path)).get("k_scan", {})
        except Exception:
            continue
        if mr and int(row.get("rows", -1)) == n and row.get("hbm_bytes_per_launch"):
            found.append((int(mr.group(1)), os.path.getmtime(path), path, row["hbm_bytes_per_launch"]))
    if not found:
        return None, None
    rnd, _, path, b = max(found)
    return b, {"file": os.path.relpath(path, ROOT), "round": rnd}


def extra_legs(lib, mq, torch, dev, stream, col, ws, ws_bytes, n, lo, hi, gold, cpu=True) -> dict:
    """Secondary measurements (rank 0, N=1): the API path with positions
    materialized (config 2's 4N+4K), and config 3 (select col0 -> fetch col1 ->
    avg) both as the three-operator chain and fused."""
    sp = mq.stream_of(stream)
    out = {}
    with torch.cuda.stream(stream):
        pos = torch.empty(n, dtype=torch.int32, device=dev)
        cnt = torch.zeros(1, dtype=torch.int64, device=dev)
        col1 = torch.empty(n, dtype=torch.int32, device=dev)
        mq.check(lib.mq_gen_uniform(col1.data_ptr(), n, 43, n, sp), "gen")
        agg = torch.zeros(4, dtype=torch.int64, device=dev)

        def timed(fn, reps=10):
            for _ in range(2):
                fn()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            e0.record(stream)
            for _ in range(reps):
                fn()
            e1.record(stream)
            torch.cuda.synchronize()
            return e0.elapsed_time(e1) / reps

        def positions():
            mq.check(lib.mq_select_positions(col.data_ptr(), None, n, 1, lo, 1, hi, pos.data_ptr(),
                                             cnt.data_ptr(), ws.data_ptr(), ws_bytes, sp))

        nblk = C.c_uint32()

        def two_launch():  # the headline step before the in-kernel combine (A/B)
            mq.check(lib.mq_select_partials(col.data_ptr(), n, 1, lo, 1, hi, 0, ws.data_ptr(),
                                            ws_bytes, C.byref(nblk), sp))
            mq.check(lib.mq_combine_partials(ws.data_ptr(), nblk.value, agg.data_ptr(), sp))

        def one_launch():
            mq.check(lib.mq_select_sum(col.data_ptr(), n, 1, lo, 1, hi, agg.data_ptr(),
                                       ws.data_ptr(), ws_bytes, sp))

        out["headline_ab"] = {"ms_two_launch": timed(two_launch, 20),
                              "ms_one_launch": timed(one_launch, 20),
                              "note": "k_scan + k_final vs k_scan with in-kernel combine, "
                                      "back-to-back on one stream"}
        t_pos = timed(positions)
        k = int(cnt.item())
        vals = torch.empty(max(k, 1), dtype=torch.int32, device=dev)

        def chain():
            positions()
            mq.check(lib.mq_fetch(col1.data_ptr(), pos.data_ptr(), k, vals.data_ptr(), sp))
            mq.check(lib.mq_reduce(vals.data_ptr(), k, agg.data_ptr(), ws.data_ptr(), ws_bytes, sp))

        t_chain = timed(chain)
        a = agg.cpu()
        c3 = [r for r in gold["config3"] if r["n"] == n]
        chain_ok = bool(c3) and (int(a[0]), int(a[1])) == (c3[0]["k"], c3[0]["sum"])

        def fused():
            mq.check(lib.mq_select_fetch_agg(col.data_ptr(), col1.data_ptr(), n, 1, lo, 1, hi,
                                             agg.data_ptr(), ws.data_ptr(), ws_bytes, sp))

        t_fused = timed(fused)
        a2 = agg.cpu()
        fused_ok = bool(c3) and (int(a2[0]), int(a2[1])) == (c3[0]["k"], c3[0]["sum"])
        out["print_positions"] = print_leg(lib, mq, torch, dev, stream, pos, k, cpu=cpu)
        out["config2_positions"] = {
            "ms": t_pos, "rows_per_s": n / (t_pos * 1e-3), "k": k,
            "algorithmic_bytes": 4 * n + 4 * k,
            "gbs_algorithmic": (4 * n + 4 * k) / (t_pos * 1e-3) / 1e9,
            "hbm_bytes_design": 4 * n + 12 * k,
            "note": "k_select_stage, one launch: 4N read; positions in an LDS ring per wave, "
                    "spilled to the workspace (4K write + 4K read) at 1 %, then 4K output write"}
        out["config3_chain"] = {
            "ms": t_chain, "rows_per_s": n / (t_chain * 1e-3), "parity": chain_ok,
            "avg": (int(a[1]) / int(a[0])) if int(a[0]) else None,
            "algorithmic_bytes": 4 * n + 12 * k}
        # the gather's line over-fetch: every match reads its
        # col1 row through a whole 64-byte line; distinct lines touched = the lines that
        # hold at least one matching row (counted from the positions, on the device)
        lines = torch.unique_consecutive(pos[:k].to(torch.int64) // 16).numel()
        out["config3_fused"] = {
            "ms": t_fused, "rows_per_s": n / (t_fused * 1e-3), "parity": fused_ok,
            "algorithmic_bytes": 4 * n + 8 * k,
            "gather_lines": lines, "gather_lines_bytes": 64 * lines,
            "gather_overfetch": (64 * lines) / (4 * k) if k else None,
            "hbm_bytes_design": 4 * n + 64 * lines,
            "gbs_design": (4 * n + 64 * lines) / (t_fused * 1e-3) / 1e9,
            "frac_design": (4 * n + 64 * lines) / (t_fused * 1e-3) / 1e9 / HBM_PEAK_GBS,
            "note": "select col0 + gather col1 at matches, one kernel (k_scan_gather: matches "
                    "staged per wave in LDS, gathered 8 loads in flight per lane); the gather reads "
                    "gather_lines 64-B lines of col1 for its 4K useful bytes"}
        out["positions_sweep"] = positions_sweep(lib, mq, torch, dev, stream, col, col1, ws, ws_bytes, n, pos, cnt,
                                                 gold)
        del pos, col1, vals
    out["config1_10m"] = config1_leg(lib, mq, torch, dev, stream, gold, cpu=cpu)
    out["shared_select"] = shared_leg(lib, mq, torch, dev, stream, col, n)
    out["config5_hash_join"] = join_leg(lib, mq, torch, dev, stream, gold, cpu=cpu)
    out["config5_many_to_many"] = join_dup_leg(lib, mq, torch, dev, stream, gold, cpu=cpu)
    out["load_csv_config3_table"] = load_leg(lib, mq, torch, dev, stream, col, n, cpu=cpu)
    out["index_build"] = index_leg(lib, mq, torch, dev, stream, col, n, cpu=cpu)
    out["pcie_probe"] = pcie_probe(torch, dev, stream)
    out["api_path_config3"] = api_leg_processes(n, lo, hi)
    return out


def config1_leg(lib, mq, torch, dev, stream, gold, cpu: bool = True) -> dict:
    """Config 1: the 10M-row column, select 1 % -> fetch -> sum. The
    reference's own query.c chain (oracle/_ref/libref.so at -O2 and libref_O0.so, the
    -O0 its Makefile builds, src/Makefile:12), median of 3 on 1 core, and the GPU step
    (mq_select_sum, HBM-resident) on the same column; K and the sum against the 10M
    golden (tests/golden/goldens.json, made by the reference)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import refcpu  # baseline / checker only
    n = 10_000_000
    lo, hi = int(0.25 * n), int(0.25 * n) + int(0.01 * n)
    want = [r for r in gold["select"] if r["n"] == n and abs(r["sel"] - 0.01) < 1e-12][0]
    sp = mq.stream_of(stream)
    res = {"n": n, "low": lo, "high": hi}
    with torch.cuda.stream(stream):
        col = torch.empty(n, dtype=torch.int32, device=dev)
        mq.check(lib.mq_gen_uniform(col.data_ptr(), n, 42, n, sp), "gen")
        ws_bytes = lib.mq_scan_workspace_bytes(n)
        ws = torch.empty(ws_bytes, dtype=torch.uint8, device=dev)
        agg = torch.zeros(4, dtype=torch.int64, device=dev)
        ms = _events_ms(torch, stream, lambda: mq.check(lib.mq_select_sum(
            col.data_ptr(), n, 1, lo, 1, hi, agg.data_ptr(), ws.data_ptr(), ws_bytes, sp), "select_sum"), 20)
        a = agg.cpu()
        res["gpu"] = {"ms": ms, "rows_per_s": n / (ms * 1e-3), "gbs": 4 * n / (ms * 1e-3) / 1e9,
                      "parity": (int(a[0]), int(a[1])) == (want["k"], want["sum"]),
                      "note": "one mq_select_sum launch (k_scan<kSum>); 40 MB is below the 256 MB "
                              "Infinity Cache, so this is a launch-latency-scale step"}
        del col, ws
    if cpu and refcpu.have_reference():
        from refapi import Api, make_column
        d = refcpu.gen_uniform(n, 42, nthreads=16)
        c = make_column(d)
        for name, path in (("reference_O2", refcpu.REFLIB), ("reference_O0", refcpu.REFLIB_O0)):
            api = Api(refcpu.reference(path))
            times, s = [], None
            for _ in range(3):
                t0 = time.perf_counter()
                pos = api.select_column(c, lo, hi)
                s = api.sum_result(api.fetch_column(c, pos))
                times.append(time.perf_counter() - t0)
            t = statistics.median(times)
            res[name] = {"ms": 1e3 * t, "rows_per_s": n / t, "cores": 1, "kind": "reference",
                         "parity": (len(pos), s) == (want["k"], want["sum"]),
                         "what": f"select_column -> fetch_column -> sum, {os.path.basename(path)}, median of 3"}
    return res


def positions_sweep(lib, mq, torch, dev, stream, col, col1, ws, ws_bytes, n, pos, cnt, gold) -> dict:
    """SURVEY §8(d) config 2's selectivity sweep through the ordered compaction
    (k_select_stage): select_column_scan's positions (query.c:92-137) and the
    select_result payload form (query.c:38-86: a match emits payload[row], here col1),
    at 0.1 / 1 / 10 / 50 / 100 % of the 1e9-row column, [N/4, N/4 + sel N). HIP events,
    median of 5. Algorithmic bytes: positions 4N + 4K; payload 4N + 4K (payload rows
    read at matches) + 4K. Parity: K and the FNV of the positions against the
    reference's goldens at 1 % and 50 % (tests/golden/goldens.json)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import refcpu  # checker only (FNV of the positions)
    sp = mq.stream_of(stream)
    res = {}
    for sel in (0.001, 0.01, 0.1, 0.5, 1.0):
        lo = int(0.25 * n)
        hi = lo + int(sel * n)
        row = {}
        for form, payload in (("positions", None), ("select_result", col1)):
            fn = lambda: mq.check(lib.mq_select_positions(  # noqa: E731
                col.data_ptr(), None if payload is None else payload.data_ptr(), n, 1, lo, 1, hi, pos.data_ptr(),
                cnt.data_ptr(), ws.data_ptr(), ws_bytes, sp), "select_positions")
            with torch.cuda.stream(stream):
                ms = _events_ms(torch, stream, fn, 5)
            k = int(cnt.item())
            ab = 4 * n + 4 * k + (4 * k if payload is not None else 0)
            row[form] = {"ms": ms, "k": k, "algorithmic_bytes": ab, "gbs": ab / (ms * 1e-3) / 1e9,
                         "frac": ab / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS}
            if payload is None:
                want = [r for r in gold["select"] if r["n"] == n and abs(r["sel"] - sel) < 1e-12]
                if want:
                    fnv = refcpu.fnv1a64(pos[:k].cpu().numpy())
                    row[form]["parity"] = (k, f"{fnv:016x}") == (want[0]["k"], want[0]["pos_fnv1a64"])
        res[f"sel_{sel:g}"] = row
    return res


def api_leg_processes(n, lo, hi, procs: int = 3) -> dict:
    """api_leg in `procs` fresh processes, one after the other (the API
    path's time varies from process to process: payload pages, helper-thread placement).
    Reports the median over the processes of each process's median, with the spread, and
    every process's record."""
    import subprocess
    runs = []
    for _ in range(procs):
        r = subprocess.run([sys.executable, os.path.abspath(__file__), "--api-child", "--rows", str(n),
                            "--lo", str(lo), "--hi", str(hi)], capture_output=True, text=True, timeout=600)
        line = [x for x in r.stdout.splitlines() if x.startswith("{")]
        if r.returncode != 0 or not line:
            runs.append({"error": f"rc={r.returncode}", "stderr_tail": r.stderr[-400:]})
            continue
        runs.append(json.loads(line[-1]))
    ok = [x for x in runs if "error" not in x]
    res = {"processes": procs, "per_process": runs}
    if ok:
        for key in ("ms_select_column", "ms_fetch_column", "ms_average", "ms_chain", "ms_free_results",
                    "d2h_payload_gbs", "ms_upload_two_columns"):
            v = [x[key] for x in ok if x.get(key) is not None]
            if v:
                res[key] = statistics.median(v)
                res[key + "_spread"] = [min(v), max(v)]
        res["k"] = ok[0]["k"]
        res["avg"] = ok[0]["avg"]
        res["parity"] = all(x.get("parity") is True for x in ok) and len(ok) == procs
        res["note"] = ("median over the processes of each process's median of 4 reps (spread = min, max of "
                       "the process medians); " + ok[0]["note"])
    else:
        res["parity"] = False
    return res


def api_child(args) -> None:
    """One api_leg process (bench.py --api-child): libmq through ctypes, no torch."""
    mq = _load("mq_binding", os.path.join(PKG, "mq.py"))
    lib = mq.load()
    mq.check(lib.mq_init(0), "mq_init")
    gold = json.load(open(os.path.join(ROOT, "tests", "golden", "goldens.json")))
    print(json.dumps(api_leg(lib, mq, args.rows, args.lo, args.hi, gold)), flush=True)


def api_leg(lib, mq, n, lo, hi, gold) -> dict:
    """Config 3 through the drop-in C API as the reference server calls it
    (server.c:137-247): host Columns (malloc'd like the mmap'd column files),
    select_column(col0) -> fetch_column(col1, positions) -> average, Result*
    handed from call to call. Reports the PCIe-inclusive times: the one-off H2D
    of each 4 GB column (column residency), then the chain on resident columns,
    whose results come back to host memory as the reference's API requires."""
    import numpy as np
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import refcpu  # input generator only (the §8(c) column, on the host)
    from refapi import make_column, _libc
    import mmap
    maps = []

    def file_column(seed):
        # the reference keeps columns in MAP_SHARED file mappings (start_data,
        # db_manager.c:736-790); a memfd is such a file, so libmq can guard it and
        # keep its HBM copy across operators
        fd = os.memfd_create(f"col{seed}")
        os.ftruncate(fd, 4 * n)
        m = mmap.mmap(fd, 4 * n, mmap.MAP_SHARED, mmap.PROT_READ | mmap.PROT_WRITE)
        os.close(fd)
        a = np.frombuffer(m, dtype=np.int32)
        refcpu.lib().rc_gen_uniform(a.ctypes.data, n, seed, n, host_cores()[0])
        maps.append(m)
        return a

    c0, c1 = file_column(42), file_column(43)
    col0, col1 = make_column(c0, b"col0"), make_column(c1, b"col1")
    # the process's first staged upload also creates the pinned staging ring and the
    # copy threads: a 64 MB column takes that one-off cost before the timed uploads
    warm = np.arange(1 << 24, dtype=np.int32)
    wcol = make_column(warm, b"warm")
    mq.check(lib.mq_column_upload(C.byref(wcol)), "upload warm-up")
    lib.mq_column_invalidate(C.byref(wcol))
    t0 = time.perf_counter()
    mq.check(lib.mq_column_upload(C.byref(col0)), "upload col0")
    mq.check(lib.mq_column_upload(C.byref(col1)), "upload col1")
    t_up = time.perf_counter() - t0
    lo_c, hi_c = C.c_int(lo), C.c_int(hi)
    times = {"select_column": [], "fetch_column": [], "average": [], "free_results": []}
    xfers = []
    avg = None
    k = 0
    for rep in range(5):
        st = mq.Status(0, None)
        lib.mq_transfer_seconds(1)
        t0 = time.perf_counter()
        rp = lib.select_column(C.byref(col0), C.byref(lo_c), C.byref(hi_c), C.byref(st))
        t1 = time.perf_counter()
        rf = lib.fetch_column(C.byref(col1), rp, C.byref(st))
        t2 = time.perf_counter()
        ra = lib.average(rf, C.byref(st))
        t3 = time.perf_counter()
        assert st.code == mq.OK
        xfer = lib.mq_transfer_seconds(0)
        k = rp.contents.num_tuples
        avg = C.cast(ra.contents.payload, C.POINTER(C.c_double))[0]
        t4 = time.perf_counter()
        for r in (rp, rf, ra):
            _libc.free(r.contents.payload)
            _libc.free(r)
        t5 = time.perf_counter()
        if rep:
            times["select_column"].append(t1 - t0)
            times["fetch_column"].append(t2 - t1)
            times["average"].append(t3 - t2)
            times["free_results"].append(t5 - t4)
            xfers.append((xfer, t3 - t0))
    med = {f"ms_{name}": 1e3 * statistics.median(v) for name, v in times.items()}
    chain_s = (med["ms_select_column"] + med["ms_fetch_column"] + med["ms_average"]) / 1e3
    # transfer share of the same reps: the median rep by chain time, its D2H seconds
    # (counted from an idle stream, so kernels are not in them)
    xfers.sort(key=lambda x: x[1])
    x_med, wall_med = xfers[len(xfers) // 2]
    want = next((r for r in gold["config3"] if r["n"] == n and r["low"] == lo and r["high"] == hi), None)
    resid = mq.residency(lib)
    lib.mq_release_all()
    res = {"rows": n, "k": k, "avg": avg, "ms_upload_two_columns": 1e3 * t_up,
           "residency": {"column_uploads": resid["column_uploads"], "guards_live": resid["guards_live"],
                         "result_uploads": resid["result_uploads"]},
           "upload_gbs": 8.0 * n / t_up / 1e9, **med, "ms_chain": 1e3 * chain_s,
           "rows_per_s_chain": n / chain_s, "ms_transfer_median_chain": 1e3 * x_med,
           "ms_wall_median_chain": 1e3 * wall_med,
           "d2h_payload_gbs": 8.0 * k / x_med / 1e9 if x_med > 0 else None,
           "note": "PCIe-inclusive: each operator returns malloc'd host payloads (client_context.c "
                   "frees them; ms_free_results is that free, outside the chain); the chain runs on "
                   "HBM-resident columns after the one-off upload (memfd-backed columns, write-guarded); "
                   "ms_transfer_median_chain and ms_wall_median_chain come from the same rep"}
    if want is not None:
        res["parity"] = (k, avg) == (want["k"], want["avg"])
    return res


def shared_leg(lib, mq, torch, dev, stream, col, n) -> dict:
    """S11 shared_select on the 1e9-row column: Q range queries of 0.1 % each,
    count + write (the host gets the counts in between, as the query API does) vs Q
    separate ordered selects; outputs allocated once, medians of repeated runs."""
    import numpy as np
    sp = mq.stream_of(stream)
    res = {}
    rng = np.random.default_rng(5)
    for q in (2, 16, 150):
        lows = rng.integers(0, n - n // 1000, q).astype(np.int32)
        highs = (lows + n // 1000).astype(np.int32)
        lo_c = (C.c_int32 * q)(*lows.tolist())
        hi_c = (C.c_int32 * q)(*highs.tolist())
        wsb = lib.mq_shared_select_workspace_bytes(n, q)
        with torch.cuda.stream(stream):
            ws = torch.empty(wsb, dtype=torch.uint8, device=dev)
            k = (C.c_uint64 * q)()
            # one untimed call sizes the outputs (the caller's allocation is not the
            # operator's work) and takes the first-call setup; then count + write,
            # median of 5, each ending in a device sync
            mq.check(lib.mq_shared_select_count(col.data_ptr(), n, lo_c, hi_c, q, k, ws.data_ptr(), wsb, sp))
            outs = [torch.empty(max(int(x), 1), dtype=torch.int32, device=dev) for x in k]
            ptrs = (C.c_void_p * q)(*[o.data_ptr() for o in outs])
            mq.check(lib.mq_shared_select_write(ws.data_ptr(), ptrs, sp))
            ts = []
            for _ in range(5):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                mq.check(lib.mq_shared_select_count(col.data_ptr(), n, lo_c, hi_c, q, k, ws.data_ptr(), wsb, sp))
                mq.check(lib.mq_shared_select_write(ws.data_ptr(), ptrs, sp))
                torch.cuda.synchronize()
                ts.append(time.perf_counter() - t0)
            t1 = statistics.median(ts)
            # the same with q separate ordered selects (median of 3)
            sws = lib.mq_scan_workspace_bytes(n)
            ws2 = torch.empty(sws, dtype=torch.uint8, device=dev)
            cnt = torch.zeros(1, dtype=torch.int64, device=dev)
            one = torch.empty(n, dtype=torch.int32, device=dev)  # capacity n: any K fits
            ts = []
            for _ in range(3):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for j in range(q):
                    mq.check(lib.mq_select_positions(col.data_ptr(), None, n, 1, int(lows[j]), 1, int(highs[j]),
                                                     one.data_ptr(), cnt.data_ptr(), ws2.data_ptr(), sws, sp))
                torch.cuda.synchronize()
                ts.append(time.perf_counter() - t0)
            t2 = statistics.median(ts)
            # parity: every query's K and positions equal the ordered select's (itself
            # pinned to the 1e9 goldens), compared on the device
            ok = True
            for j in range(q):
                mq.check(lib.mq_select_positions(col.data_ptr(), None, n, 1, int(lows[j]), 1, int(highs[j]),
                                                 one.data_ptr(), cnt.data_ptr(), ws2.data_ptr(), sws, sp))
                kj = int(cnt.item())
                ok = ok and kj == int(k[j]) and torch.equal(outs[j][:kj], one[:kj])
            del outs, one, ws, ws2
        res[f"q{q}"] = {"ms_shared": 1e3 * t1, "ms_q_separate_selects": 1e3 * t2,
                        "rows_x_queries_per_s": n * q / t1, "k_total": int(sum(k)), "parity": bool(ok)}
    return res


def join_leg(lib, mq, torch, dev, stream, gold, logn: int = 28, cpu: bool = True) -> dict:
    """Config 5: 2^28 x 2^28 hash join (build + probe + pair write), keys of
    SURVEY.md §8(c); parity = M and the FNV-1a-64 of the pairs vs the reference."""
    import numpy as np
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import refcpu  # checker only (pair hash)
    n = 1 << logn
    sp = mq.stream_of(stream)
    with torch.cuda.stream(stream):
        a = torch.empty(n, dtype=torch.int32, device=dev)
        b = torch.empty(n, dtype=torch.int32, device=dev)
        p = torch.empty(n, dtype=torch.int32, device=dev)
        mq.check(lib.mq_gen_join_keys(a.data_ptr(), n, 0, sp))
        mq.check(lib.mq_gen_join_keys(b.data_ptr(), n, 1, sp))
        mq.check(lib.mq_gen_iota(p.data_ptr(), n, sp))
        times, m = [], 0
        o1 = o2 = None
        for rep in range(4):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            h = C.c_void_p()
            mq.check(lib.mq_join_build(a.data_ptr(), p.data_ptr(), n, C.byref(h), sp), "join_build")
            mm = C.c_uint64()
            mq.check(lib.mq_join_probe(h, b.data_ptr(), n, C.byref(mm), sp), "join_probe")
            m = mm.value
            if o1 is None:
                o1 = torch.empty(m, dtype=torch.int32, device=dev)
                o2 = torch.empty(m, dtype=torch.int32, device=dev)
            mq.check(lib.mq_join_write(h, p.data_ptr(), o1.data_ptr(), o2.data_ptr(), sp))
            torch.cuda.synchronize()
            times.append(time.perf_counter() - t0)
            mq.check(lib.mq_join_free(h))
        t = statistics.median(times[1:])
        want = [r for r in gold["join_survey"] if r["n"] == n]
        fnv = refcpu.fnv1a64_pairs(o1.cpu().numpy(), o2.cpu().numpy())
        ok = bool(want) and (m, f"{fnv:016x}") == (want[0]["m"], want[0]["pairs_fnv1a64"])
        del a, b, p, o1, o2
        # the probe's random-access ceiling: n random 8-byte reads of a table of the
        # join's size (2^(logn+1) slots), k_ht_probe_unique's pattern without compares
        tbl = torch.zeros(1 << (logn + 1), dtype=torch.int64, device=dev)
        wsr = torch.empty(1, dtype=torch.int64, device=dev)
        ceil_ms = _events_ms(torch, stream, lambda: mq.check(
            lib.mq_random_read(tbl.data_ptr(), logn + 1, n, wsr.data_ptr(), sp), "random_read"), 5)
        del tbl
    res = {"n_build": n, "n_probe": n, "m": m, "ms": 1e3 * t,
           "random_read_ceiling": {"kernel": "k_random_read", "reads": n, "table_bytes": 8 << (logn + 1),
                                   "ms": ceil_ms, "g_reads_per_s": n / ceil_ms / 1e6,
                                   "note": "n random 8-byte slot reads = the probe's table traffic; "
                                           "k_ht_probe_unique's own time is in the rocprof stats"},
           "rows_per_s": 2 * n / t, "algorithmic_bytes": 8 * n + 8 * n + 8 * m,
           "gbs_algorithmic": (16 * n + 8 * m) / t / 1e9, "parity": ok,
           "note": "wall time of build+probe+write incl. 2 host syncs (dup flag, M); "
                   "unique-key build path (keys are a bijection)"}
    if cpu and refcpu.have_reference():  # the reference's own join, at a size it finishes quickly
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        from refapi import Api
        api = Api(refcpu.reference())
        k = 1 << 20
        ka, kb, kp = refcpu.gen_join(k, "build"), refcpu.gen_join(k, "probe"), refcpu.gen_join(k, "iota")
        t0 = time.perf_counter()
        api.join(ka, kp, kb, kp, "hash")
        tr = time.perf_counter() - t0
        res["cpu_reference_2e20"] = {"s": tr, "rows_per_s": 2 * k / tr, "cores": 1,
                                     "kind": "reference"}
    if cpu:
        res["cpu_host_cores_2e24"] = host_cores_join(refcpu, gold, "build", "probe", gold["join_survey"])
    return res


def host_cores_join(refcpu, gold, kb: str, kp: str, rows: list, logn: int = 24) -> dict:
    """Config 5's host-cores baseline: the restatement's hash join
    over every core this process may use (rc_hash_join_mt: partitioned build, range-split
    probe; output identical to the reference's), median of 3 at 2^logn x 2^logn, with M
    and the pair FNV checked against the reference's golden."""
    import numpy as np
    n = 1 << logn
    cores, why = host_cores()
    a, b, p = refcpu.gen_join(n, kb), refcpu.gen_join(n, kp), refcpu.gen_join(n, "iota")
    want = [r for r in rows if r["n"] == n]
    m = want[0]["m"] if want else n * 2
    o1, o2 = np.empty(m, dtype=np.int32), np.empty(m, dtype=np.int32)
    L = refcpu.lib()
    times, got = [], 0
    for _ in range(3):
        t0 = time.perf_counter()
        got = L.rc_hash_join_mt(refcpu._a(a), refcpu._a(p), n, refcpu._a(b), refcpu._a(p), n, refcpu._a(o1),
                                refcpu._a(o2), m, cores)
        times.append(time.perf_counter() - t0)
    t = statistics.median(times)
    ok = bool(want) and got == m and f"{refcpu.fnv1a64_pairs(o1, o2):016x}" == want[0]["pairs_fnv1a64"]
    return {"n_build": n, "n_probe": n, "m": int(got), "s": t, "rows_per_s": 2 * n / t, "cores": cores,
            "cores_from": why, "kind": "port", "parity": ok,
            "what": "oracle/refcpu.c rc_hash_join_mt (keys " + kb + " x " + kp + "), median of 3"}


def join_dup_leg(lib, mq, torch, dev, stream, gold, logn: int = 28, cpu: bool = True) -> dict:
    """Config 5, many-to-many: every build key twice (rows i and
    i + n/2), about half the probes hit, two matches each (M ~ n): the duplicate-key
    build path (stable radix sort into key runs). Parity: M and the pair FNV at 2^22
    against the reference's own hash_join (tests/golden/make_join_dup_goldens.py);
    timing at 2^logn (build + probe + write, as join_leg). Parity at 2^24 (round 6)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import refcpu  # checker only (pair hash)
    sp = mq.stream_of(stream)

    def run(n, keep):
        with torch.cuda.stream(stream):
            a = torch.empty(n, dtype=torch.int32, device=dev)
            b = torch.empty(n, dtype=torch.int32, device=dev)
            p = torch.empty(n, dtype=torch.int32, device=dev)
            mq.check(lib.mq_gen_join_keys(a.data_ptr(), n, 2, sp))
            mq.check(lib.mq_gen_join_keys(b.data_ptr(), n, 3, sp))
            mq.check(lib.mq_gen_iota(p.data_ptr(), n, sp))
            times, m, o1, o2 = [], 0, None, None
            for rep in range(4 if not keep else 1):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                h = C.c_void_p()
                mq.check(lib.mq_join_build(a.data_ptr(), p.data_ptr(), n, C.byref(h), sp), "join_build")
                mm = C.c_uint64()
                mq.check(lib.mq_join_probe(h, b.data_ptr(), n, C.byref(mm), sp), "join_probe")
                m = mm.value
                if o1 is None:
                    o1 = torch.empty(max(m, 1), dtype=torch.int32, device=dev)
                    o2 = torch.empty(max(m, 1), dtype=torch.int32, device=dev)
                mq.check(lib.mq_join_write(h, p.data_ptr(), o1.data_ptr(), o2.data_ptr(), sp))
                torch.cuda.synchronize()
                times.append(time.perf_counter() - t0)
                mq.check(lib.mq_join_free(h))
            out = (m, statistics.median(times[1:]) if len(times) > 1 else times[0])
            if keep:
                out += (refcpu.fnv1a64_pairs(o1[:m].cpu().numpy(), o2[:m].cpu().numpy()),)
            del a, b, p, o1, o2
            return out

    want = [r for r in gold.get("join_dup", []) if r["n"] == 1 << 24]
    pm, _, pf = run(1 << 24, True)
    ok = bool(want) and (pm, f"{pf:016x}") == (want[0]["m"], want[0]["pairs_fnv1a64"])
    n = 1 << logn
    m, t = run(n, False)
    res = {"n_build": n, "n_probe": n, "m": m, "ms": 1e3 * t, "rows_per_s": 2 * n / t,
           "algorithmic_bytes": 16 * n + 8 * m, "gbs_algorithmic": (16 * n + 8 * m) / t / 1e9,
           "parity_2e24": ok, "note": "wall time incl. the duplicate-key sample, the partition of the "
                                      "build rows and 2 host syncs; the window join answers duplicate "
                                      "keys (k_win_join_runs, DESIGN §3.3 round 6)"}
    if cpu and refcpu.have_reference():
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        from refapi import Api
        api = Api(refcpu.reference())
        k = 1 << 20
        ka, kb, kp = refcpu.gen_join(k, "build_dup"), refcpu.gen_join(k, "probe_dup"), refcpu.gen_join(k, "iota")
        t0 = time.perf_counter()
        api.join(ka, kp, kb, kp, "hash")
        tr = time.perf_counter() - t0
        res["cpu_reference_2e20"] = {"s": tr, "rows_per_s": 2 * k / tr, "cores": 1, "kind": "reference"}
    if cpu:
        res["cpu_host_cores_2e24"] = host_cores_join(refcpu, gold, "build_dup", "probe_dup", gold.get("join_dup", []))
    return res


def _events_ms(torch, stream, fn, reps):
    """Median of reps timed calls (HIP events on the launch stream) after one warm-up."""
    ms = []
    for i in range(reps + 1):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(stream)
        fn()
        b.record(stream)
        b.synchronize()
        if i:
            ms.append(a.elapsed_time(b))
    return statistics.median(ms)


def load_leg(lib, mq, torch, dev, stream, col, n, cpu: bool = True) -> dict:
    """SURVEY 8(f) row 1, the load path: config 3's table (4 int32 columns of n rows,
    seeds 42..45) as CSV text in HBM (mq_format_csv_int32, "v,v,v,v\n" rows), then
    load_db's data loop on the GPU: mq_csv_count_rows + mq_csv_parse_int32 (events).
    Parity: every parsed column equals its source. CPU: the reference's own load_db
    (oracle/_ref/libdbm.so) on the first 2M rows of the same text."""
    import numpy as np
    sp = mq.stream_of(stream)
    ncols = 4
    with torch.cuda.stream(stream):
        cols = [col] + [torch.empty(n, dtype=torch.int32, device=dev) for _ in range(ncols - 1)]
        for j in range(1, ncols):
            mq.check(lib.mq_gen_uniform(cols[j].data_ptr(), n, 42 + j, n, sp), "gen")
        fws = torch.empty(lib.mq_format_csv_workspace_bytes(n, ncols), dtype=torch.uint8, device=dev)
        text = torch.empty(n * ncols * 11 + 16, dtype=torch.uint8, device=dev)
        ptrs = (C.c_void_p * ncols)(*[c.data_ptr() for c in cols])
        nb = C.c_uint64()
        mq.check(lib.mq_format_csv_int32(ptrs, ncols, n, text.data_ptr(), C.byref(nb), fws.data_ptr(),
                                         fws.numel(), sp), "format_csv")
        del fws
        tb = nb.value
        ws = torch.empty(lib.mq_csv_workspace_bytes(tb, ncols), dtype=torch.uint8, device=dev)
        outs = [torch.empty(n, dtype=torch.int32, device=dev) for _ in range(ncols)]
        optrs = (C.c_void_p * ncols)(*[o.data_ptr() for o in outs])
        mm = torch.empty(2 * ncols, dtype=torch.int32, device=dev)
        rows = C.c_uint64()
        count = lambda: mq.check(lib.mq_csv_count_rows(text.data_ptr(), tb, ncols, C.byref(rows),  # noqa: E731
                                                       ws.data_ptr(), ws.numel(), sp), "csv_count")
        parse = lambda: mq.check(lib.mq_csv_parse_int32(text.data_ptr(), tb, ncols, optrs, rows.value,  # noqa: E731
                                                        mm.data_ptr(), ws.data_ptr(), ws.numel(), sp),
                                 "csv_parse")
        ms_count = _events_ms(torch, stream, count, 3)
        ms_parse = _events_ms(torch, stream, parse, 3)
        ok = rows.value == n and all(torch.equal(o, c) for o, c in zip(outs, cols))
        sample = None
        head = text[: min(tb, 2_000_000 * ncols * 11)].cpu().numpy().tobytes()
        del outs, ws, text, cols[1:]
    t = (ms_count + ms_parse) * 1e-3
    res = {"rows": n, "ncols": ncols, "text_bytes": tb, "ms_count": ms_count, "ms_parse": ms_parse,
           "rows_per_s": n / t, "text_gbs": tb / t / 1e9,
           "hbm_bytes_design": 2 * tb + 4 * n * ncols,
           "gbs_design": (2 * tb + 4 * n * ncols) / t / 1e9, "parity": bool(ok),
           "note": "count pass (streaming '\\n' count, 1 read of the text) + parse pass (LDS-staged, "
                   "SWAR tokens, 1 read + 4 B per cell written)"}
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import refload  # the reference's load_db, baseline only
    if cpu and refload.have():
        import tempfile
        cut = head.rfind(b"\n", 0, len(head)) + 1
        sample = head[:cut]
        srows = sample.count(b"\n")
        with tempfile.TemporaryDirectory() as tmp:
            path = os.path.join(tmp, "t.csv")
            with open(path, "wb") as f:
                f.write((",".join(f"db.tbl.c{j}" for j in range(ncols)) + "\n").encode() + sample)
            r = refload.load(path, ncols)
        res["cpu_reference"] = {"rows": srows, "s": r["load_s"], "rows_per_s": srows / r["load_s"],
                                "cores": 1, "kind": "reference",
                                "what": "load_db + insert_row (libdbm.so, gcc -O2), incl. table growth"}
    return res


def exact_index_leg(lib, mq, torch, dev, stream, logn: int = 27) -> dict:
    """build_index's exact path at its size limit: the §8(c)
    uniform column of 2^27 rows (seed 42, values in [0, 2^27): 49M tied neighbours),
    sorted in the reference quicksort's own order. ms_lomuto = mq_index_build_lomuto
    (the level-synchronous Lomuto restatement, one host sync per recursion depth);
    ms_build_index = mq_index_build_ref as build_index runs it (radix sort, tie
    check, then the Lomuto restatement); ms_radix = the radix sort alone. Parity: the
    FNV of values and positions equal the goldens the reference's own quicksort made
    (tests/golden/quicksort_goldens.json)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import refcpu  # checker only (FNV)
    n = 1 << logn
    sp = mq.stream_of(stream)
    gold = [c for c in json.load(open(os.path.join(ROOT, "tests", "golden", "quicksort_goldens.json")))
            if c["n"] == n and c["seed"] == 42 and c["modulus"] == n]
    with torch.cuda.stream(stream):
        c = torch.empty(n, dtype=torch.int32, device=dev)
        mq.check(lib.mq_gen_uniform(c.data_ptr(), n, 42, n, sp), "gen")
        v = torch.empty(n, dtype=torch.int32, device=dev)
        p = torch.empty(n, dtype=torch.int64, device=dev)
        ms_radix = _events_ms(torch, stream, lambda: mq.check(
            lib.mq_index_build(c.data_ptr(), n, v.data_ptr(), p.data_ptr(), sp), "index_build"), 2)
        ms_lomuto = _events_ms(torch, stream, lambda: mq.check(
            lib.mq_index_build_lomuto(c.data_ptr(), n, v.data_ptr(), p.data_ptr(), sp), "lomuto"), 2)
        ok_l = bool(gold) and (f"{refcpu.fnv1a64(v.cpu().numpy()):016x}", f"{refcpu.fnv1a64(p.cpu().numpy()):016x}") == \
            (gold[0]["values_fnv"], gold[0]["positions_fnv"])
        ex = C.c_int(-1)
        ms_ref = _events_ms(torch, stream, lambda: mq.check(
            lib.mq_index_build_ref(c.data_ptr(), n, v.data_ptr(), p.data_ptr(), n, C.byref(ex), sp), "ref"), 2)
        ok_r = bool(gold) and ex.value == 1 and \
            (f"{refcpu.fnv1a64(v.cpu().numpy()):016x}", f"{refcpu.fnv1a64(p.cpu().numpy()):016x}") == \
            (gold[0]["values_fnv"], gold[0]["positions_fnv"])
        del c, v, p
    return {"rows": n, "ms_lomuto": ms_lomuto, "ms_build_index": ms_ref, "ms_radix": ms_radix,
            "rows_per_s_build_index": n / (ms_ref * 1e-3), "parity": ok_l and ok_r,
            "ties": gold[0]["ties"] if gold else None,
            "path": "exact tie order (the reference quicksort's), as build_index applies it up to 2^27 rows"}


def index_leg(lib, mq, torch, dev, stream, col, n, cpu: bool = True) -> dict:
    """the sorted index of the 1e9-row column (mq_index_build:
    stable radix sort of (value, row) -> values + size_t positions; MSD levels and an
    LDS finisher at this size, csrc/mq_isort.hip). Parity: gather
    through the positions reproduces the values (and they ascend). CPU: the
    reference's quicksort (index.c:25-46, libdbm.so) on 1e6 rows of the same column."""
    import numpy as np
    sp = mq.stream_of(stream)
    with torch.cuda.stream(stream):
        v = torch.empty(n, dtype=torch.int32, device=dev)
        p = torch.empty(n, dtype=torch.int64, device=dev)
        ms = _events_ms(torch, stream, lambda: mq.check(
            lib.mq_index_build(col.data_ptr(), n, v.data_ptr(), p.data_ptr(), sp), "index_build"), 2)
        g = torch.empty(n, dtype=torch.int32, device=dev)
        mq.check(lib.mq_gather_u64(col.data_ptr(), p.data_ptr(), n, g.data_ptr(), sp))
        ok = bool(torch.equal(g, v)) and bool((v[1:] >= v[:-1]).all())
        del v, p, g
    res = {"rows": n, "ms": ms, "rows_per_s": n / (ms * 1e-3), "parity": ok,
           "hbm_bytes_design": 58 * n,
           "path": "mq_index_build: the stable radix sort alone (equal values in ascending row order); "
                   "its MSD form (csrc/mq_isort.hip) at this size and key range",
           "note": "min/max (4N), two MSD levels of 256 range-proportional digits (histogram 4N / 1N, "
                   "scatter 4N+9N / 8N+8N), LDS counting finisher (8N read, 12N written) = 58 B a row; "
                   "the 4-pass LSD form (MQ_INDEX_SORT=lsd4) moves 74"}
    res["exact_2e27"] = exact_index_leg(lib, mq, torch, dev, stream)
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import refload  # the reference's quicksort, baseline only
    if cpu and refload.have():
        k = 1_000_000
        vals = col[:k].cpu().numpy().astype(np.int32).copy()
        pos = np.arange(k, dtype=np.uint64)
        L = C.CDLL(refload.LIBDBM)
        L.quicksort.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_int]
        t0 = time.perf_counter()
        L.quicksort(vals.ctypes.data, pos.ctypes.data, 0, k - 1)
        tq = time.perf_counter() - t0
        res["cpu_reference"] = {"rows": k, "s": tq, "rows_per_s": k / tq, "cores": 1,
                                "kind": "reference", "what": "quicksort (index.c:25-46, libdbm.so -O2)"}
    return res


if __name__ == "__main__":
    main()
