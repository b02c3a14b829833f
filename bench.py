#!/usr/bin/env python3
"""bench.py — headline benchmark of mpigx (BASELINE.json metric:
"Allreduce! busbw GB/s (256MiB f32 SUM) at 1/2/4/8 GPUs; % of xGMI/HBM peak").

  python bench.py [--gpus N --steps K --warmup W]            (N = 1)
  python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N

N = 1 runs BASELINE config 2 — the single-GPU form of the metric: the device
MPI.Op kernel reduces 8 rank buffers of 256 MiB f32 with SUM in HBM
(mpigx_reduce_local_multi, MPICH association).  One step = one kernel launch
over the 8 x 256 MiB inputs; value = algorithmic HBM GB/s (9 x 256 MiB per
step / wall time per step), roofline against HBM.

N > 1 runs config 3 at 256 MiB: MPI.Allreduce!(SUM) of 256 MiB f32 per rank,
blocking MPI semantics; value = busbw = S/t * 2(N-1)/N (nccl-tests), the max
time over ranks, roofline against aggregate xGMI ingress.  The same line
carries the Allreduce size sweep, the RCCL comparison, config 4
(Bcast!/Allgather!/Alltoall! sweep), config 5 (Scan!/Exscan!/Reduce! on
Int32/Int64 with BAND/BOR/MAX, bit-exact check) and the reference path
(MPICH MPI_Allreduce, 8 ranks on the host cores) measured in the same run.

Rank 0 prints ONE JSON line.  Inputs are synthetic, resident in HBM before
timing.
"""
import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "mpi.jl_amd"))
sys.path.insert(0, ROOT)

HBM_PEAK_GBPS = 8000.0  # MI355X_MICROARCH.md chip table (spec); 6.29 TB/s measured float4 copy
XGMI_LINK_GBPS = 76.8   # per direction: 153.6 GB/s bidirectional per xGMI link (MI355X spec), 7 links


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--mib", type=int, default=256)
    p.add_argument("--nbuf", type=int, default=8)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-iters", type=int, default=30)
    p.add_argument("--no-rccl", action="store_true", help="skip the RCCL comparison (N>1)")
    p.add_argument("--no-extra", action="store_true", help="skip the config-4/5 blocks (N>1)")
    p.add_argument("--no-sweep", action="store_true",
                   help="N=1: skip the size sweep (rocprof runs, so the headline kernel's stats hold 256 MiB launches only)")
    return p.parse_args()


def cpu_baseline_local(nbuf, mib, iters):
    """MPICH 3.3.2 MPI_Reduce_local over the same workload (oracle/_ref)."""
    exe = os.path.join(ROOT, "oracle", "_ref", "mpich_bench")
    if os.path.exists(exe):
        out = subprocess.run([exe, "local", str(nbuf), str(mib), str(iters)], capture_output=True, text=True,
                             timeout=600)
        line = [l for l in out.stdout.splitlines() if l.startswith("{")]
        if out.returncode == 0 and line:
            j = json.loads(line[-1])
            return {"value": round(j["algo_GBps"], 3), "unit": "GB/s", "cores": 1, "kind": "reference",
                    "sample": f"MPICH 3.3.2 MPI_Reduce_local, {nbuf} x {mib} MiB f32 SUM, full workload, "
                              f"{iters} timed calls (+1 warm-up), 1 thread",
                    "sec_per_step": j["sec_per_call"]}
    # fallback: the numpy port (oracle) on a 1/8 sample
    import numpy as np
    from oracle import mpich_model as M
    cnt = (mib << 18) // 8
    ins = [np.random.default_rng(k).uniform(-1, 1, cnt).astype(np.float32) for k in range(nbuf)]
    t0 = time.perf_counter()
    for _ in range(3):
        M.fold_rsag(ins, "FLOAT", "SUM")
    t = (time.perf_counter() - t0) / 3
    return {"value": round((nbuf + 1) * cnt * 4 / t / 1e9, 3), "unit": "GB/s", "cores": 1, "kind": "port",
            "sample": f"numpy oracle, {nbuf} x {mib // 8} MiB f32 SUM, 3 calls"}


def host_cpu():
    model = ""
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return {"host_threads": os.cpu_count(), "usable_threads": len(os.sched_getaffinity(0)), "model": model}


def cpu_reference_allreduce(ranks=8, mib=256, iters=3):
    """The reference path on the host cores: MPICH 3.3.2 MPI_Allreduce(f32 SUM)
    under `mpiexec -n ranks` (oracle/_ref/mpich_bench; the call MPI.jl makes at
    collective.jl:698-700)."""
    exe = os.path.join(ROOT, "oracle", "_ref", "mpich_bench")
    mpiexec = "/opt/conda/bin/mpiexec"
    if not (os.path.exists(exe) and os.path.exists(mpiexec)):
        return {"error": "MPICH harness not built (oracle/Makefile) or mpiexec missing"}
    try:
        out = subprocess.run([mpiexec, "-n", str(ranks), exe, "allreduce", str(mib), str(iters)],
                             capture_output=True, text=True, timeout=300)
    except subprocess.TimeoutExpired:
        return {"error": "timeout"}
    line = [l for l in out.stdout.splitlines() if l.startswith("{")]
    if out.returncode != 0 or not line:
        return {"error": (out.stderr or out.stdout)[-200:]}
    j = json.loads(line[-1])
    return {"ranks": ranks, "cores": min(ranks, os.cpu_count() or ranks), "mib": mib, "iters": iters,
            "sec_per_call": j["sec_per_call"], "algbw_GBps": j["algbw_GBps"], "busbw_GBps": j["busbw_GBps"],
            "kind": "reference", "impl": "MPICH 3.3.2 MPI_Allreduce f32 SUM, host buffers", **host_cpu()}


def cpu_reference_sweep(ranks=8, maxmib=256):
    """BASELINE.md's CPU plan in the same run: MPICH 3.3.2 under `mpiexec -n
    ranks` on the host cores — Allreduce f32 SUM at the GPU sweep's sizes,
    Bcast / Allgather / Alltoall at config 4's, Scan / Exscan / Reduce
    Int32/Int64 BAND/BOR/MAX at 1 Ki / 1 Mi / 16 Mi elements (config 5's
    64 Mi bounded: MPICH's Scan moves ~0.1 GB/s per rank), called like
    collective.jl's ccall sites (oracle/mpich_bench.c `sweep`)."""
    exe = os.path.join(ROOT, "oracle", "_ref", "mpich_bench")
    mpiexec = "/opt/conda/bin/mpiexec"
    if not (os.path.exists(exe) and os.path.exists(mpiexec)):
        return {"error": "MPICH harness not built (oracle/Makefile) or mpiexec missing"}
    t0 = time.perf_counter()
    try:
        out = subprocess.run([mpiexec, "-n", str(ranks), exe, "sweep", str(maxmib)], capture_output=True, text=True,
                             timeout=400)
    except subprocess.TimeoutExpired:
        return {"error": "timeout"}
    line = [l for l in out.stdout.splitlines() if l.startswith("{")]
    if out.returncode != 0 or not line:
        return {"error": (out.stderr or out.stdout)[-200:]}
    j = json.loads(line[-1])
    j.update({"cores": min(ranks, os.cpu_count() or ranks), "kind": "reference", "impl": "MPICH 3.3.2, host buffers",
              "wall_s": round(time.perf_counter() - t0, 1), **host_cpu()})
    return j


def cpu_baseline_from_allreduce(cpu_ar):
    """The N > 1 line's cpu_baseline: the reference path itself — MPICH 3.3.2
    MPI_Allreduce(f32 SUM) of the same per-rank size over 8 ranks on this
    box's host cores (the call behind /root/reference/src/collective.jl:
    698-700), measured in the same run (cpu_reference_allreduce), as busbw in
    the headline's unit.  None when that run failed or was skipped."""
    if not cpu_ar or "busbw_GBps" not in cpu_ar:
        return None
    return {"value": round(cpu_ar["busbw_GBps"], 3), "unit": "GB/s (busbw)", "cores": cpu_ar["cores"],
            "kind": "reference", "model": cpu_ar.get("model", ""),
            "sample": f"MPICH 3.3.2 MPI_Allreduce f32 SUM, {cpu_ar['mib']} MiB per rank, {cpu_ar['ranks']} ranks "
                      f"(mpiexec) on the host cores, {cpu_ar['iters']} timed calls, host buffers, full workload",
            "sec_per_step": cpu_ar["sec_per_call"], "algbw_GBps": cpu_ar.get("algbw_GBps")}


def traffic_from_profiles(key):
    """(per-launch HBM bytes, file) from the newest committed PMC pass
    (profiles/r<NN>*_traffic.json, tools/profile.sh: rocprofv3 cannot run
    inside the process it profiles)."""
    import glob
    best, src = None, None
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "*traffic*.json"))):
        try:
            j = json.load(open(f))
        except Exception:
            continue
        if key in j:
            best, src = j[key], os.path.relpath(f, ROOT)
    return best, src


def coll_hbm_bytes(kind, n, S):
    """Algorithmic HBM bytes of one S-byte Allreduce, all n ranks on one GPU
    (tools/coll_prof.py algo_bytes): pull two-shot S(2 + (n-1)/n) per rank,
    pull-push 2S, push 2S(1 + (n-1)/n)."""
    if kind == "pullpush":
        return 2 * n * S
    if kind == "push":
        return 2 * n * S * (1 + (n - 1) / n)
    return n * S * (2 + (n - 1) / n)


def coll_traffic_from_profiles(kind, n, mib):
    """(HBM bytes of one call, all ranks, file) from the newest committed
    collective-kernel PMC profile (profiles/r<NN>*_coll_n<n>_1gpu*.json,
    tools/coll_prof.py, whatever its suffix: _xdev_fullgrid etc.).  Files
    sort by their round prefix; the last one holding this (size, variant)
    wins."""
    import glob
    best, src = None, None
    files = glob.glob(os.path.join(ROOT, "profiles", f"*_coll_n{n}_1gpu*.json"))
    for f in sorted(files, key=os.path.basename):
        try:
            t = json.load(open(f))["configs"].get(f"{mib}:{kind}", {}).get("traffic") or {}
        except Exception:
            continue
        for k, v in t.items():
            # rank 0's kernel HBM bytes (round 4's key; tools/coll_prof.py
            # names it hbm_bytes_device since round 5)
            b = v.get("hbm_bytes_rank0", v.get("hbm_bytes_device"))
            if "ar_zc_kernel" in k and b:
                best, src = b * n, os.path.relpath(f, ROOT)
    return best, src


def bench_local(args):
    import torch
    import mpigx as MPI

    cpu = None if args.no_cpu_baseline else cpu_baseline_local(args.nbuf, args.mib, args.cpu_iters)
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    count = args.mib << 18
    S = count * 4
    g = torch.Generator(device=dev).manual_seed(1234)
    ins = [(torch.rand(count, device=dev, generator=g) * 2 - 1) for _ in range(args.nbuf)]
    out = torch.empty(count, device=dev)
    stream = torch.cuda.current_stream(dev)

    def step():
        MPI.reduce_local_multi(ins, out, MPI.SUM, stream=stream)

    # the box's own ceiling for this kernel: a read-only
    # stream of the same 8 inputs in the fold's access layout, no fold, no
    # stores (mpigx_read_probe, copy.hip read_probe_kernel), HIP-event timed on
    # the same stream; MI355X boxes differ in HBM read rate by ~8 %
    # (profiles/r02_fold_tune_box*.json), so roofline.frac_vs_measured is the
    # number that is comparable from box to box
    import ctypes
    sink = torch.zeros(4096, dtype=torch.uint8, device=dev)
    in_ptrs = (ctypes.c_void_p * len(ins))(*[x.data_ptr() for x in ins])

    def read_probe_ms(reps=10):
        L = MPI.lib()
        for _ in range(2):
            MPI.api._check(L.mpigx_read_probe(in_ptrs, len(ins), S, ctypes.c_void_p(sink.data_ptr()),
                                              ctypes.c_void_p(stream.cuda_stream)))
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(stream)
        for _ in range(reps):
            L.mpigx_read_probe(in_ptrs, len(ins), S, ctypes.c_void_p(sink.data_ptr()), ctypes.c_void_p(stream.cuda_stream))
        b.record(stream)
        torch.cuda.synchronize()
        return a.elapsed_time(b) / reps

    # the fold's own mix: the same 8 reads plus the
    # 256 MiB of write-through stores, XOR in place of the fold
    # (mpigx_mix_probe, copy.hip mix_probe_kernel) — the ceiling that is
    # this kernel's own; the read-only rate stays beside it
    def mix_probe_ms(reps=10):
        L = MPI.lib()
        for _ in range(2):
            MPI.api._check(L.mpigx_mix_probe(in_ptrs, len(ins), S, ctypes.c_void_p(out.data_ptr()),
                                             ctypes.c_void_p(stream.cuda_stream)))
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(stream)
        for _ in range(reps):
            L.mpigx_mix_probe(in_ptrs, len(ins), S, ctypes.c_void_p(out.data_ptr()), ctypes.c_void_p(stream.cuda_stream))
        b.record(stream)
        torch.cuda.synchronize()
        return a.elapsed_time(b) / reps

    # everything beside the headline is guarded: a section that raises is
    # recorded in `errors` and the headline line is still printed
    errors = {}

    def guarded(name, fn, default=None):
        try:
            return fn()
        except Exception as e:  # noqa: BLE001
            errors[name] = f"{type(e).__name__}: {str(e)[:200]}"
            torch.cuda.synchronize()
            return default

    probes = len(ins) in (1, 2, 4, 8)
    read_ms = guarded("read_probe", lambda: [read_probe_ms()], []) if probes else []
    mix_ms = guarded("mix_probe", lambda: [mix_probe_ms()], []) if probes else []
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    # the timed K steps: wall clock for `value`; HIP events on the launch
    # stream bracketing the same K back-to-back launches give the kernel's
    # average launch duration for the roofline (no per-launch instrumentation)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record(stream)
    for _ in range(args.steps):
        step()
    e1.record(stream)
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / args.steps
    kern_ms = e0.elapsed_time(e1) / args.steps
    algo = (args.nbuf + 1) * S
    if read_ms:
        read_ms += guarded("read_probe", lambda: [read_probe_ms()], [])
    if mix_ms:
        mix_ms += guarded("mix_probe", lambda: [mix_probe_ms()], [])

    # parity spot check (the probes above wrote `out`: one more fold first)
    step()
    torch.cuda.synchronize()
    # parity spot check of the timed output vs the MPICH-pinned oracle (1 Mi elements)
    import numpy as np
    from oracle import mpich_model as M
    k = 1 << 20
    sample = [x[:k].cpu().numpy() for x in ins]
    ref = M.fold_rsag(sample, "FLOAT", "SUM")
    # the whole-buffer schedule is the Rabenseifner regime; its per-element
    # association does not depend on count, so a prefix sample is exact
    parity = bool(np.array_equal(out[:k].cpu().numpy().view(np.uint32), ref.view(np.uint32)))

    # secondary variants (same kernel family), kernel time only
    def time_variant(dtype_, op):
        xs = [x.to(dtype_) for x in ins] if dtype_ != torch.float32 else ins
        o = torch.empty(count, device=dev, dtype=dtype_)
        for _ in range(2):
            MPI.reduce_local_multi(xs, o, op, stream=stream)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(5):
            MPI.reduce_local_multi(xs, o, op, stream=stream)
        e1.record(stream)
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 5
        return round((args.nbuf + 1) * count * xs[0].element_size() / (ms / 1e3) / 1e9, 1)

    def time_in_place(k):
        """f32 SUM written over rank buffer k (out aliases input k: MPI_Reduce
        / Allreduce IN_PLACE, MPI_Reduce_local's inoutbuf), on a copy of that
        input: the same 9 x 256 MiB of traffic with one stream fewer, the
        store landing in a DRAM row the thread has just read
        (tools/mix_tune.hip)."""
        xs = list(ins)
        xs[k] = ins[k].clone()
        for _ in range(2):
            MPI.reduce_local_multi(xs, xs[k], MPI.SUM, stream=stream)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(5):
            MPI.reduce_local_multi(xs, xs[k], MPI.SUM, stream=stream)
        e1.record(stream)
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 5
        del xs
        return round((args.nbuf + 1) * count * 4 / (ms / 1e3) / 1e9, 1)

    variants = guarded("variants", lambda: {
        "f32_MAX_GBps": time_variant(torch.float32, MPI.MAX),
        "bf16_SUM_GBps": time_variant(torch.bfloat16, MPI.SUM),
        "bf16_MAX_GBps": time_variant(torch.bfloat16, MPI.MAX),
        "f32_SUM_in_place_rank0_GBps": time_in_place(0),
        f"f32_SUM_in_place_rank{args.nbuf - 1}_GBps": time_in_place(args.nbuf - 1)}, {})

    # message-size sweep of the same kernel (f32 SUM, 8 inputs), HIP events
    # over back-to-back launches: "us" issued through the Python mirror,
    # "us_abi" through the raw C ABI, "us_graph" replayed from one captured
    # HIP graph (device-bound: below ~4 MiB the eager loops measure the host
    # issuing launches, not the kernel)
    sweep = {}
    def sweep_point(mib):
        k = mib << 18
        xs = [x[:k] for x in ins]
        o = out[:k]
        for _ in range(3):
            MPI.reduce_local_multi(xs, o, MPI.SUM, stream=stream)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        reps = 20
        e0.record(stream)
        for _ in range(reps):
            MPI.reduce_local_multi(xs, o, MPI.SUM, stream=stream)
        e1.record(stream)
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / reps * 1e3
        # the same loop through the raw C ABI (what MPI.jl's ccall makes: no
        # Python mirror between launches)
        Lr, pin = MPI.lib(), (ctypes.c_void_p * len(xs))(*[x.data_ptr() for x in xs])
        po, ps, fl, sm = ctypes.c_void_p(o.data_ptr()), ctypes.c_void_p(stream.cuda_stream), MPI.FLOAT.val, MPI.SUM.val
        e0.record(stream)
        for _ in range(reps):
            Lr.mpigx_reduce_local_multi(pin, len(xs), po, k, fl, sm, 0, ps)
        e1.record(stream)
        torch.cuda.synchronize()
        us_abi = e0.elapsed_time(e1) / reps * 1e3
        # the same launches replayed from one captured HIP graph: the host's
        # per-launch cost out of the loop (below ~4 MiB the eager loop above
        # is bound by the host issuing launches, not by the kernel)
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            for _ in range(reps):
                MPI.reduce_local_multi(xs, o, MPI.SUM)
        graph.replay()
        torch.cuda.synchronize()
        usg = 1e9
        for _ in range(3):  # best of three replays (a single replay catches box noise)
            e0.record(stream)
            graph.replay()
            e1.record(stream)
            torch.cuda.synchronize()
            usg = min(usg, e0.elapsed_time(e1) / reps * 1e3)
        del graph
        sweep[f"{mib}MiB"] = {"GBps": round((args.nbuf + 1) * k * 4 / (us / 1e6) / 1e9, 1), "us": round(us, 2),
                              "us_abi": round(us_abi, 2),
                              "GBps_graph": round((args.nbuf + 1) * k * 4 / (usg / 1e6) / 1e9, 1),
                              "us_graph": round(usg, 2),
                              "frac_hbm_graph": round((args.nbuf + 1) * k * 4 / (usg / 1e6) / 1e9 / HBM_PEAK_GBPS, 4)}

    for mib in (() if args.no_sweep else (1, 4, 16, 64)):
        guarded(f"sweep_{mib}MiB", lambda: sweep_point(mib))
    sweep[f"{args.mib}MiB"] = {"GBps": round(algo / (kern_ms / 1e3) / 1e9, 1), "us": round(kern_ms * 1e3, 2),
                               "frac_hbm": round(algo / (kern_ms / 1e3) / 1e9 / HBM_PEAK_GBPS, 4)}
    cpu_ar = None if args.no_cpu_baseline else cpu_reference_allreduce()

    traffic, traffic_src = traffic_from_profiles("reduce_local_multi_f32_sum_8x256MiB")
    print(json.dumps(build_local_line({
        "nbuf": args.nbuf, "mib": args.mib, "steps": args.steps, "warmup": args.warmup, "wall_s": wall,
        "kern_ms": kern_ms, "read_ms": read_ms, "mix_ms": mix_ms, "parity": parity, "variants": variants,
        "sweep": sweep, "cpu": cpu, "cpu_ar": cpu_ar, "traffic": traffic, "traffic_src": traffic_src,
        "errors": errors})), flush=True)


def build_local_line(m):
    """The N = 1 JSON line from the measured sections (m: bench_local's
    numbers; tests/test_bench_line_cpu.py builds it from recorded ones)."""
    S = m["mib"] << 20
    algo = (m["nbuf"] + 1) * S
    achieved = algo / (m["kern_ms"] / 1e3) / 1e9
    value = algo / m["wall_s"] / 1e9
    # the box's ceilings: the faster of the two probes of each kind (before /
    # after the timed steps).  peak_measured = the 8-read : 1-write mix
    # probe, the fold's own traffic with no fold; the read-only stream beside it
    mix = algo / (min(m["mix_ms"]) / 1e3) / 1e9 if m.get("mix_ms") else None
    rd = (m["nbuf"] * S) / (min(m["read_ms"]) / 1e3) / 1e9 if m.get("read_ms") else None
    return {
        "metric": "Allreduce! busbw GB/s (256MiB f32 SUM) at 1/2/4/8 GPUs; % of xGMI/HBM peak",
        "value": round(value, 2), "unit": "GB/s", "n_gpus": 1, "steps": m["steps"], "warmup": m["warmup"],
        "ms_per_step": round(m["wall_s"] * 1e3, 4), "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "dtype": "f32", "data": "synthetic (uniform[-1,1) f32, seeded, resident in HBM)",
        "config": {"workload": f"config 2: 1xMI355X local MPI.Op kernel, reduce {m['nbuf']} rank buffers of "
                               f"{m['mib']} MiB f32 SUM (MPICH association) -> 1 output",
                   "parallelism": "single GPU", "nbuf": m["nbuf"], "bytes_per_buffer": S,
                   "algorithmic_bytes_per_step": algo},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBPS, 4), "traffic": m["traffic"],
                     "peak_measured": round(mix, 1) if mix else None,
                     "frac_vs_measured": round(achieved / mix, 4) if mix else None,
                     "peak_measured_basis": "this box's 8-read : 1-write stream in the fold's layout and store "
                                            "policy (mpigx_mix_probe: the 8 x 256 MiB inputs read, their XOR "
                                            "written to the 256 MiB output with the fold's write-through stores, "
                                            "9 x 256 MiB counted), HIP events, faster of one probe before and one "
                                            "after the timed steps",
                     "peak_read_only": round(rd, 1) if rd else None,
                     "frac_vs_read_only": round(achieved / rd, 4) if rd else None,
                     "peak_read_only_basis": "mpigx_read_probe: the same 8 inputs read, nothing written (8 x 256 MiB "
                                             "counted)",
                     "kernel": "fold_local_kernel<OpSum,float,NMAX 8,TREE,SH_FULL,U 4>",
                     "kernel_ms": round(m["kern_ms"], 4),
                     "achieved_basis": "9 x 256 MiB algorithmic bytes / (HIP-event time over the K timed launches on "
                                       "the launch stream / K)",
                     "traffic_basis": "rocprofv3 PMC: 2 x FETCH_SIZE + WRITE_SIZE per dispatch (gfx950 FETCH_SIZE "
                                      f"halving, MI355X_MICROARCH.md), {m['traffic_src']}"},
        "cpu_baseline": m["cpu"],
        "parity_sample_bit_exact": m["parity"],
        "variants": m["variants"],
        "sweep_local_f32_sum": m["sweep"],
        "cpu_reference_allreduce_256MiB": m["cpu_ar"],
        "errors": m.get("errors") or None,
    }


class _StdoutToStderr:
    """Gloo prints its connection notes ("[Gloo] Rank 0 is connected to ...")
    on file descriptor 1 while a process group forms; they go to stderr so
    that rank 0's stdout holds only the one JSON line."""

    def __enter__(self):
        sys.stdout.flush()
        self.saved = os.dup(1)
        os.dup2(2, 1)

    def __exit__(self, *exc):
        sys.stdout.flush()
        os.dup2(self.saved, 1)
        os.close(self.saved)


def bench_allreduce(args):
    import ctypes

    import numpy as np
    import torch
    import torch.distributed as dist
    import mpigx as MPI
    from oracle import mpich_model as M

    t_start = time.perf_counter()
    rank = int(os.environ.get("RANK", 0))
    n = int(os.environ.get("WORLD_SIZE", 1))
    local = int(os.environ.get("LOCAL_RANK", rank)) % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    with _StdoutToStderr():
        dist.init_process_group("gloo", rank=rank, world_size=n)
        dist.barrier()  # every connection made (and noted) inside
    comm = MPI.Init()
    dev = torch.device(f"cuda:{local}")
    stream = torch.cuda.current_stream(dev)
    # same-device ranks (the 1-GPU test box) move HBM bytes through IPC, not xGMI
    buses = [None] * n
    dist.all_gather_object(buses, torch.cuda.get_device_properties(dev).pci_bus_id)
    same_device = len(set(buses)) == 1

    def tmax(*xs):
        tt = torch.tensor(list(xs), dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        return tt.tolist()

    def rank_input(q, count):
        g = torch.Generator(device=dev).manual_seed(1000 + q)
        return torch.rand(count, device=dev, generator=g) * 2 - 1

    def time_ar(nbytes, steps, warmup, fn=None, keep=False):
        """(wall s/step, device s/step) of blocking Allreduce!(SUM) f32, max over ranks."""
        count = nbytes // 4
        send = rank_input(rank, count)
        recv = torch.empty_like(send)
        call = (lambda: MPI.Allreduce_(send, recv, MPI.SUM, comm)) if fn is None else (lambda: fn(send, recv))
        # the communicator's tuners (mpigx.cpp ar_tune_* / mt_*) sample their
        # candidates on the first calls of a size: untimed, before the warmup
        for _ in range(8 if fn is None else 0):
            call()
        for _ in range(warmup):
            call()
        torch.cuda.synchronize()
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
        dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for a, b in ev:
            a.record(stream)
            call()
            b.record(stream)
        torch.cuda.synchronize()
        dist.barrier()
        wall = (time.perf_counter() - t0) / steps
        kern = sum(a.elapsed_time(b) for a, b in ev) / steps / 1e3
        w, k = tmax(wall, kern)
        return (w, k, send, recv) if keep else (w, k)

    def check_sample(recv, count, label):
        """The timed output against the MPICH-pinned oracle on a sample of every
        rank's (regenerated) random input: the prefix and the elements around
        every two-shot chunk boundary (each chunk is folded by another rank).
        The f32 SUM association is element-position independent, so sampled
        slices are exact.  Max over ranks (every rank checks its recvbuf)."""
        chunk = -(-(-(-count // n)) // 4) * 4
        spans = [(0, min(count, 1 << 20))]
        for c in range(1, n):
            spans.append((max(0, c * chunk - 4096), min(count, c * chunk + 4096)))
        spans.append((max(0, count - 4096), count))
        ok = True
        xs = [rank_input(q, count) for q in range(n)]
        for lo, hi in spans:
            ins = [x[lo:hi].cpu().numpy() for x in xs]
            ref = M.fold_rsag(ins, "FLOAT", "SUM") if hi - lo >= n else M.allreduce(ins, "FLOAT", "SUM")[0]
            ok &= bool(np.array_equal(recv[lo:hi].cpu().numpy().view(np.uint32), ref.view(np.uint32)))
        del xs
        (bad,) = tmax(0.0 if ok else 1.0)
        return {"sample_bit_exact_vs_oracle": bad == 0.0, "spans": len(spans), "label": label}

    def busbw(nbytes, t):
        return nbytes / t * 2 * (n - 1) / n / 1e9

    S = args.mib << 20
    # the communicator's large-Allreduce tuner (mpigx.cpp ar_tune_*) decides
    # between the pull, push and pull-push two-shots on its first zero-copy
    # calls (registration, then one call each: time_ar's untimed prelude)
    _ = time_ar(S, 2, 0)
    ch, costs = ctypes.c_int(-1), (ctypes.c_double * 3)()
    MPI.lib().mpigx_comm_ar_costs(comm.val, ctypes.byref(ch), costs)
    ar_tune = {"choice": {-1: "undecided", 0: "pull two-shot", 1: "push two-shot", 2: "pull-push two-shot"}[ch.value],
               "pull_ns_per_MiB": round(costs[0], 1), "push_ns_per_MiB": round(costs[1], 1),
               "pullpush_ns_per_MiB": round(costs[2], 1),
               "basis": "device time of one 256 MiB call each, max over ranks decides (rank 0's shown)"}
    t, kern, send, recv = time_ar(S, args.steps, args.warmup, keep=True)
    correct = check_sample(recv, S // 4, "timed buffers, default algorithm")
    del send, recv

    # Everything below is reported beside the headline.  A section that raises
    # (on every rank, e.g. an MPI error class returned by a variant) is
    # recorded and the later sections are skipped, so the headline line is
    # still printed.
    errors, alive = {}, [True]
    section_s = {"headline": round(time.perf_counter() - t_start, 2)}  # wall seconds per section (rank 0)

    def guarded(name, fn, default=None, engine=True):
        # engine=False: the section does not call libmpigx (RCCL), so it runs
        # even after an engine section broke the communicator
        if engine and not alive[0]:
            errors[name] = "skipped after an earlier failure"
            return default
        t_sec = time.perf_counter()
        try:
            out, bad = fn(), 0.0
        except Exception as e:  # noqa: BLE001
            out, bad = default, 1.0
            errors[name] = f"{type(e).__name__}: {str(e)[:200]}"
        (anybad,) = tmax(bad)
        section_s[name] = round(time.perf_counter() - t_sec, 2)
        if engine and not anybad and alive[0]:  # back to the defaults (collective: every rank is here)
            MPI.set_knob(comm, "ALGO", None)
            MPI.set_knob(comm, "RING_CHANNELS", 1)
        if anybad and engine:
            alive[0] = False
        return out

    # measured xGMI ingress/egress of my GPU over the same workload (SMU
    # metrics, per link, KB; tools/xgmi_counters.py) vs the algorithmic
    # 2S(n-1)/n each way per rank and step
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import xgmi_counters as XC
    bus = torch.cuda.get_device_properties(dev).pci_bus_id

    def xgmi_section():
        c0 = XC.read(bus)
        # every rank takes the same branch: a rank whose metrics read failed
        # must not skip the collectives below while its peers wait in them
        (missing,) = tmax(1.0 if c0 is None else 0.0)
        if missing:
            return None
        reps = max(args.steps, 10)
        xs = rank_input(rank, S // 4)
        xr = torch.empty_like(xs)
        dist.barrier()
        for _ in range(reps):
            MPI.Allreduce_(xs, xr, MPI.SUM, comm)
        torch.cuda.synchronize()
        dist.barrier()
        time.sleep(0.2)  # let the metrics table refresh
        c1 = XC.read(bus)
        if c1 is None:
            return None
        rd = sum(b - a for a, b in zip(c0["read_kb"], c1["read_kb"])) * 1024 / reps
        wr = sum(b - a for a, b in zip(c0["write_kb"], c1["write_kb"])) * 1024 / reps
        algo_x = 2 * S * (n - 1) / n
        return {"read_bytes_per_step": rd, "write_bytes_per_step": wr, "algorithmic_bytes_per_step": algo_x,
                "read_over_algorithmic": round(rd / algo_x, 4), "source": "amd-smi gpu_metrics xgmi_*_data_acc",
                "steps": reps}
    xg = guarded("xgmi_counters", xgmi_section)

    # size sweep (mpigx), algorithm variants, the ring (MPIGX_ALGO=ring, one
    # ring / every coprime-stride ring) and the RCCL comparison point
    sweep, rccl = {}, {}
    # config 3's sweep: every power of two from 8 KiB to 1 GiB,
    # busbw and its fraction of the nominal aggregate xGMI ingress (distinct
    # GPUs; null when the ranks share one GPU)
    sizes = [(8 << 10) << k for k in range(18)]
    if S not in sizes:
        sizes.append(S)
    peak_x = None if same_device else XGMI_LINK_GBPS * (n - 1)

    def label(nb):
        return f"{nb >> 10}KiB" if nb < (1 << 20) else f"{nb >> 20}MiB"

    def sweep_section():
        for nb in sizes:
            tw, tk = time_ar(nb, 5 if nb >= (256 << 20) else 10, 2)
            sweep[label(nb)] = {"busbw": round(busbw(nb, tw), 1), "busbw_dev": round(busbw(nb, tk), 1),
                                "algbw": round(nb / tw / 1e9, 1), "ms": round(tw * 1e3, 4),
                                "frac_xgmi": round(busbw(nb, tk) / peak_x, 4) if peak_x else None}
        # ring reduce-scatter + allgather against the default (config 3's
        # "ring vs tree/direct"), 1 MiB .. 1 GiB
        MPI.set_knob(comm, "ALGO", "ring")
        for nb in [nb for nb in sizes if nb >= (1 << 20)]:
            tw, tk = time_ar(nb, 5 if nb >= (256 << 20) else 10, 2)
            sweep[f"ring_{label(nb)}"] = {"busbw": round(busbw(nb, tw), 1), "busbw_dev": round(busbw(nb, tk), 1),
                                          "frac_xgmi": round(busbw(nb, tk) / peak_x, 4) if peak_x else None}
        MPI.set_knob(comm, "ALGO", None)
        for nb in (1 << 20, 16 << 20):
            for algo in ("oneshot", "twoshot"):
                MPI.set_knob(comm, "ALGO", algo)
                tw, _ = time_ar(nb, 10, 2)
                sweep[f"{nb >> 20}MiB_{algo}"] = round(busbw(nb, tw), 1)
            MPI.set_knob(comm, "ALGO", None)
        # small / medium messages, every algorithm forced (the LL step, the LL
        # two-shot, the staged one-/two-shot): per-call latency in microseconds
        # (where "ll2" does not fit a chunk into half an LL slot it runs the
        # static choice)
        for nb in (8 << 10, 64 << 10, 256 << 10, 1 << 20):
            for algo in ("ll", "ll2", "oneshot", "twoshot"):
                if algo == "ll" and nb > (256 << 10):
                    continue  # beyond the LL area's capacity
                MPI.set_knob(comm, "ALGO", algo)
                tw, _ = time_ar(nb, 20, 5)
                sweep[f"{nb >> 10}KiB_{algo}_us"] = round(tw * 1e6, 2)
            MPI.set_knob(comm, "ALGO", None)
        # the engine's own per-call latency on the default path: K back-to-back
        # calls through the raw C ABI (what MPI.jl's ccall makes), no events and
        # no Python mirror in the loop, max over ranks
        for nb in (8, 8 << 10, 64 << 10):
            cnt = max(1, nb // 4)
            xs, xr = rank_input(rank, cnt), torch.empty(cnt, device=dev)
            ps, pr = ctypes.c_void_p(xs.data_ptr()), ctypes.c_void_p(xr.data_ptr())
            Lr, fl, sm, cvv = MPI.lib(), MPI.FLOAT.val, MPI.SUM.val, comm.val
            for _ in range(30):
                Lr.mpigx_allreduce(ps, pr, cnt, fl, sm, cvv)
            dist.barrier()
            reps = 300
            t0 = time.perf_counter()
            for _ in range(reps):
                Lr.mpigx_allreduce(ps, pr, cnt, fl, sm, cvv)
            (tw,) = tmax((time.perf_counter() - t0) / reps)
            sweep[f"{nb >> 10}KiB_raw_abi_us" if nb >= 1024 else f"{nb}B_raw_abi_us"] = round(tw * 1e6, 2)
        rings = len(M.ring_strides(n, 4))
        for algo, chans in (("pull", 1), ("pull_generic", 1), ("push", 1), ("pullpush", 1), ("ring", 1),
                            ("ring", rings)):
            MPI.set_knob(comm, "ALGO", algo)
            MPI.set_knob(comm, "RING_CHANNELS", chans)
            tag = algo if algo != "ring" or chans == 1 else f"ring{chans}"
            for nb in (16 << 20, S, 1 << 30):
                tw, _ = time_ar(nb, 5 if nb >= (256 << 20) else 10, 2)
                sweep[f"{nb >> 20}MiB_{tag}"] = round(busbw(nb, tw), 1)
            # the variant's timed output, checked like the default's
            _, _, s_, r_ = time_ar(S, 1, 1, keep=True)
            sweep[f"{tag}_correct"] = check_sample(r_, S // 4, f"{tag} timed buffers")["sample_bit_exact_vs_oracle"] \
                if algo != "ring" else _ring_check(M, np, r_, S // 4, n, rank_input, tmax, chans)
            del s_, r_
        MPI.set_knob(comm, "ALGO", None)
        MPI.set_knob(comm, "RING_CHANNELS", 1)
    guarded("sweep", sweep_section)
    # what the small/medium tuner chose per size class of the sweep
    tune_classes = {}

    def tune_report(kind, name, nb, names, dest):
        k = nb.bit_length() - 1
        ch, ns = ctypes.c_int(-1), (ctypes.c_double * 4)()
        MPI.lib().mpigx_comm_tune_class(comm.val, k + 64 * kind, ctypes.byref(ch), ns)
        dest[f"{name}_{nb >> 10}KiB"] = {
            "choice": "static" if ch.value < 0 else names[ch.value],
            "ns_per_MiB": {names[v]: round(ns[v], 1) for v in range(len(names))}}
    for nb in (8 << 10, 64 << 10, 256 << 10, 1 << 20):
        tune_report(0, "allreduce", nb, ("LL", "one-shot", "two-shot", "LL two-shot"), tune_classes)

    def rccl_section():
        if args.no_rccl:
            rccl["skipped"] = True
        elif same_device:
            rccl["skipped"] = "ranks share one GPU (RCCL needs one GPU per rank)"
        else:
            try:
                with _StdoutToStderr():
                    ng = dist.new_group(backend="nccl")
                for nb in sizes:
                    tw, _ = time_ar(nb, 5 if nb >= (256 << 20) else 10, 2,
                                    fn=lambda s_, r_: (r_.copy_(s_), dist.all_reduce(r_, group=ng)))
                    rccl[f"{nb >> 10}KiB" if nb < (1 << 20) else f"{nb >> 20}MiB"] = round(busbw(nb, tw), 1)
            except Exception as e:  # noqa: BLE001
                rccl["error"] = str(e)[:200]
    guarded("rccl", rccl_section, engine=False)

    # measured xGMI: every rank pulls 64 MiB from every peer at once / from one peer
    def probe_section():
        probe = {}
        for kind, name in ((0, "all_peers"), (1, "one_link")):
            secs = ctypes.c_double(0)
            pb = 64 << 20
            for _ in range(2):  # warm, then timed
                rc = MPI.lib().mpigx_comm_probe(comm.val, kind, pb, ctypes.byref(secs))
                if rc:
                    raise RuntimeError(f"mpigx_comm_probe returned {rc}")
            (sec,) = tmax(secs.value)
            probe[name + "_GBps"] = round(pb * ((n - 1) if kind == 0 else 1) / sec / 1e9, 1)
        return probe
    probe = guarded("xgmi_probe", probe_section, {})

    # where the headline call's time goes: per-block phase timestamps of the
    # kernel (mpigx_comm_set_stamps, 100 MHz device clock) on one more call of
    # each two-shot variant at the headline size; median over blocks of each
    # phase, and the span from the first block's entry to the last block's exit
    def phases_section():
        out = {}
        st = torch.zeros(1024 * 8, dtype=torch.int64, device=dev)
        xs = rank_input(rank, S // 4)
        xr = torch.empty_like(xs)
        names = ("entry_barrier", "reduce_scatter", "mid_barrier", "allgather", "exit_barrier")
        for algo in ("pull", "pull_generic", "push", "pullpush"):
            MPI.set_knob(comm, "ALGO", algo)
            for _ in range(2):
                MPI.Allreduce_(xs, xr, MPI.SUM, comm)
            st.zero_()
            MPI.lib().mpigx_comm_set_stamps(comm.val, ctypes.c_void_p(st.data_ptr()))
            MPI.Allreduce_(xs, xr, MPI.SUM, comm)
            torch.cuda.synchronize()
            MPI.lib().mpigx_comm_set_stamps(comm.val, None)
            t = st.view(1024, 8)[:, :6].cpu().numpy().astype(np.int64)
            t = t[t[:, 0] > 0]
            d = np.diff(t, axis=1) / 100.0  # us
            rec = {nm: round(float(np.median(d[:, k])), 2) for k, nm in enumerate(names)}
            rec["blocks"] = int(t.shape[0])
            rec["span_us"] = round(float(t[:, 5].max() - t[:, 0].min()) / 100.0, 2)
            rec["reduce_scatter_max_us"] = round(float(d[:, 1].max()), 2)
            rec["allgather_max_us"] = round(float(d[:, 3].max()), 2)
            out[algo] = rec
        MPI.set_knob(comm, "ALGO", None)
        del xs, xr, st
        return out
    phases = guarded("phases", phases_section, {})

    def time_call(call, steps, warmup, prelude=0):
        for _ in range(prelude + warmup):  # prelude: the tuners' sampling calls
            call()
        torch.cuda.synchronize()
        dist.barrier()
        t0 = time.perf_counter()
        for _ in range(steps):
            call()
        torch.cuda.synchronize()
        (tw,) = tmax((time.perf_counter() - t0) / steps)
        return tw

    # config 4: Bcast! / Allgather! / Alltoall! f32 sweep (S = per-rank buffer
    # for Bcast, total recv for Allgather, total send for Alltoall); busbw
    # factors as nccl-tests: 1, (n-1)/n, (n-1)/n
    cfg4 = {}
    def config4_section():
        if not args.no_extra:
            for nb in (64 << 10, 1 << 20, 16 << 20, 128 << 20, 512 << 20):
                cnt = nb // 4
                steps = 10 if nb <= (16 << 20) else 3
                buf = torch.full((cnt,), float(rank), device=dev)
                tb = time_call(lambda: MPI.Bcast_(buf, 0, comm), steps, 2, 6)
                okb = bool(torch.all(buf == 0).item())
                tbs = None
                if nb >= (128 << 20) and n >= 3:
                    # the pull scatter + allgather the zero-copy relay replaced
                    MPI.set_knob(comm, "BCAST", "sag")
                    buf.fill_(float(rank))
                    tbs = time_call(lambda: MPI.Bcast_(buf, 0, comm), steps, 1)
                    okb &= bool(torch.all(buf == 0).item())
                    MPI.set_knob(comm, "BCAST", None)
                per = cnt // n
                src = torch.full((per,), float(rank), device=dev)
                dst = torch.empty(per * n, device=dev)
                tg = time_call(lambda: MPI.Allgather_(src, dst, per, comm), steps, 2, 6)
                okg = bool(torch.equal(dst, torch.arange(n, device=dev, dtype=torch.float32).repeat_interleave(per)))
                a2s = torch.arange(n, device=dev, dtype=torch.float32).repeat_interleave(per) + 100 * rank
                a2r = torch.empty_like(a2s)
                ta = time_call(lambda: MPI.Alltoall_(a2s, a2r, per, comm), steps, 2, 6)
                oka = bool(torch.equal(a2r, torch.arange(n, device=dev, dtype=torch.float32).repeat_interleave(per) * 100
                                       + rank))
                f = (n - 1) / n
                (bad,) = tmax(0.0 if (okb and okg and oka) else 1.0)
                cfg4[f"{nb >> 10}KiB"] = {
                    "bcast_busbw": round(nb / tb / 1e9, 2), "allgather_busbw": round(nb / tg / 1e9 * f, 2),
                    "alltoall_busbw": round(nb / ta / 1e9 * f, 2), "ok": bad == 0.0}
                if peak_x:  # fraction of the nominal aggregate xGMI ingress (distinct GPUs)
                    cfg4[f"{nb >> 10}KiB"].update(
                        bcast_frac_xgmi=round(nb / tb / 1e9 / peak_x, 4),
                        allgather_frac_xgmi=round(nb / tg / 1e9 * f / peak_x, 4),
                        alltoall_frac_xgmi=round(nb / ta / 1e9 * f / peak_x, 4))
                if tbs:
                    cfg4[f"{nb >> 10}KiB"]["bcast_sag_busbw"] = round(nb / tbs / 1e9, 2)
                del buf, src, dst, a2s, a2r
    guarded("config4", config4_section)
    # the byte movers' tuner at config 4's smallest sizes (per-rank block)
    tune_classes4 = {}
    for nb, kinds in (((64 << 10), ((1, "bcast"),)), ((64 << 10) // n, ((2, "allgather"), (3, "alltoall")))):
        for kind, name in kinds:
            tune_report(kind, name, nb, ("LL", "staged"), tune_classes4)

    # config 5: Scan! / Exscan! / Reduce! with BAND/BOR/MAX on Int32/Int64,
    # bit-exact against the fold of every rank's (regenerated) input
    cfg5, cfg5_ok = {}, [True]
    def config5_section():
        # its own, shorter device timeout: a stall here fails this section in
        # 20 s instead of the default 60 s (every earlier number is printed anyway)
        MPI.lib().mpigx_comm_set_timeout(comm.val, 20000)
        try:
            config5_body()
        finally:
            MPI.lib().mpigx_comm_set_timeout(comm.val, int(os.environ.get("MPIGX_TIMEOUT_MS", 60000)))

    def config5_body():
        if not args.no_extra:
            ops = (("BAND", MPI.BAND, torch.bitwise_and), ("BOR", MPI.BOR, torch.bitwise_or),
                   ("MAX", MPI.MAX, torch.maximum))
            for tdt, lim in ((torch.int32, 1 << 31), (torch.int64, 1 << 62)):
                for cnt in (1 << 10, 1 << 20, 64 << 20):
                    def gen(q):
                        g = torch.Generator(device=dev).manual_seed(7000 + 31 * q + cnt)
                        return torch.randint(-lim, lim, (cnt,), dtype=tdt, device=dev, generator=g)
                    xs = [gen(q) for q in range(n)]
                    mine = xs[rank]
                    for oname, op, fn in ops:
                        pref = [xs[0]]
                        for q in range(1, n):
                            pref.append(fn(pref[-1], xs[q]))
                        out = torch.zeros_like(mine)
                        steps = 3 if cnt >= (64 << 20) else 5
                        res = {}
                        ts = time_call(lambda: MPI.Scan_(mine, out, op, comm), steps, 1)
                        ok = bool(torch.equal(out, pref[rank]))
                        res["scan_algbw"] = round(cnt * mine.element_size() / ts / 1e9, 2)
                        out.zero_()
                        te = time_call(lambda: MPI.Exscan_(mine, out, op, comm), steps, 1)
                        ok &= rank == 0 or bool(torch.equal(out, pref[rank - 1]))
                        res["exscan_algbw"] = round(cnt * mine.element_size() / te / 1e9, 2)
                        root = n - 1
                        rout = torch.zeros_like(mine) if rank == root else None
                        tr = time_call(lambda: MPI.Reduce_(mine, rout, op, root, comm), steps, 1)
                        if rank == root:
                            ok &= bool(torch.equal(rout, pref[-1]))
                        res["reduce_algbw"] = round(cnt * mine.element_size() / tr / 1e9, 2)
                        (bad,) = tmax(0.0 if ok else 1.0)
                        res["bit_exact"] = bad == 0.0
                        cfg5_ok[0] &= res["bit_exact"]
                        cfg5[f"{str(tdt)[6:]}_{oname}_{cnt}"] = res
                    del xs, pref, mine, out
    guarded("config5", config5_section)

    # the reference path on this box's host cores, same run (rank 0 only):
    # the headline Allreduce at 8 ranks (cpu_baseline) and at this run's
    # rank count, and BASELINE.md's whole CPU plan at 8 ranks
    cpu_ar = cpu_ar_n = cpu_sweep = None
    if not args.no_cpu_baseline:
        if rank == 0:
            cpu_ar = cpu_reference_allreduce(8, args.mib, 3)
            if n != 8:
                cpu_ar_n = cpu_reference_allreduce(n, args.mib, 3)
            cpu_sweep = cpu_reference_sweep(8, args.mib)
        dist.barrier()

    if rank == 0:
        kind = {"pull-push two-shot": "pullpush", "push two-shot": "push"}.get(ar_tune["choice"], "pull")
        traffic, traffic_src = coll_traffic_from_profiles(kind, n, args.mib) if same_device else (None, None)
        print(json.dumps(build_coll_line({
            "n": n, "mib": args.mib, "steps": args.steps, "warmup": args.warmup, "t": t, "kern": kern,
            "same_device": same_device, "ar_tune": ar_tune, "traffic": traffic, "traffic_src": traffic_src,
            "xg": xg, "cpu_ar": cpu_ar, "cpu_ar_n": cpu_ar_n, "cpu_sweep": cpu_sweep, "correct": correct, "tune_classes": tune_classes, "probe": probe,
            "phases": phases, "section_s": section_s, "sweep": sweep, "rccl": rccl, "cfg4": cfg4,
            "tune_classes4": tune_classes4, "cfg5": cfg5, "cfg5_ok": cfg5_ok[0] and "config5" not in errors,
            "errors": errors})), flush=True)
    try:
        MPI.Finalize()
    finally:
        dist.destroy_process_group()


def build_coll_line(m):
    """The N > 1 JSON line from the measured sections (m: bench_allreduce's
    numbers; tests/test_bench_line_cpu.py builds it from recorded ones)."""
    n, S, t, kern = m["n"], m["mib"] << 20, m["t"], m["kern"]

    def busbw(nbytes, tt):
        return nbytes / tt * 2 * (n - 1) / n / 1e9

    value = busbw(S, t)
    ach = busbw(S, kern)
    peak_nom = XGMI_LINK_GBPS * (n - 1)
    xg = m["xg"]
    if m["same_device"]:
        # every rank's kernel streams the same HBM: achieved = the chosen
        # variant's algorithmic HBM bytes of one call, all ranks, / device time
        kind = {"pull-push two-shot": "pullpush", "push two-shot": "push"}.get(m["ar_tune"]["choice"], "pull")
        hbm_b = coll_hbm_bytes(kind, n, S)
        roof = {"bound": "hbm (same-device IPC)", "achieved": round(hbm_b / kern / 1e9, 1), "peak": HBM_PEAK_GBPS,
                "unit": "GB/s", "frac": round(hbm_b / kern / 1e9 / HBM_PEAK_GBPS, 4), "traffic": m["traffic"],
                "kernel": f"ar_zc_kernel ({kind})", "algorithmic_hbm_bytes_per_call": hbm_b,
                "busbw_device_GBps": round(ach, 1),
                "traffic_basis": f"rocprofv3 PMC of rank 0's kernel x {n} ranks, {m['traffic_src']}"
                if m["traffic_src"] else None,
                "note": "all ranks share one GPU: peer pulls / pushes are HBM accesses through IPC mappings, no xGMI"}
    else:
        roof = {"bound": "xgmi", "achieved": round(ach, 1), "peak": round(peak_nom, 1), "unit": "GB/s",
                "frac": round(ach / peak_nom, 4),
                "traffic": xg["read_bytes_per_step"] if xg else None,
                "peak_basis": f"nominal {n - 1} links x {XGMI_LINK_GBPS} GB/s per direction (MI355X spec)"}
    roof.update({"achieved_basis": ("algorithmic HBM bytes of one call (all ranks) / " if m["same_device"] else
                                    "busbw of ")
                 + "the blocking call's device time (HIP events around each call on the comm stream), max over ranks",
                 "xgmi_traffic": xg})
    return {
        "metric": "Allreduce! busbw GB/s (256MiB f32 SUM) at 1/2/4/8 GPUs; % of xGMI/HBM peak",
        "value": round(value, 2), "unit": "GB/s", "n_gpus": n, "steps": m["steps"], "warmup": m["warmup"],
        "ms_per_step": round(t * 1e3, 4), "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "dtype": "f32", "data": "synthetic (uniform[-1,1) f32 per rank, seeded, resident in HBM)",
        "config": {"workload": f"config 3 at {m['mib']} MiB: MPI.Allreduce!(SUM) f32, blocking, {n} ranks",
                   "parallelism": f"{n} ranks x 1 GPU (hipIpc peer-mapped HBM over xGMI)"
                   if not m["same_device"] else f"{n} ranks sharing one GPU (same-device IPC)",
                   "bytes_per_rank": S, "algbw_GBps": round(S / t / 1e9, 2), "same_device_ranks": m["same_device"]},
        "roofline": roof,
        # the reference path itself on this box's host cores, same run
        # (VERDICT r05 item 1): MPICH MPI_Allreduce, 8 ranks, same size
        "cpu_baseline": cpu_baseline_from_allreduce(m["cpu_ar"]),
        "cpu_reference_allreduce": m["cpu_ar"],
        "cpu_reference_allreduce_same_ranks": m.get("cpu_ar_n"),
        "cpu_reference_sweep_8ranks": m.get("cpu_sweep"),
        "correct": m["correct"],
        "ar_tune": m["ar_tune"],
        "tune_classes": m["tune_classes"],
        "xgmi_probe_informational": dict(m["probe"] or {}, note="engine's own all-peer / one-link pull of 64 MiB; "
                                                                "not a peak (it measured below the collective at n=3 "
                                                                "in r02)"),
        "phases_headline_us": m["phases"],
        "section_wall_s": m["section_s"],
        "sweep_mpigx_busbw": m["sweep"],
        "rccl_busbw": m["rccl"],
        "config4_bcast_allgather_alltoall": m["cfg4"],
        "tune_classes_after_config4": m["tune_classes4"],
        "config5_scan_exscan_reduce": {"bit_exact_all": m["cfg5_ok"], "cases": m["cfg5"]},
        "errors": m["errors"] or None,
    }


def _ring_check(M, np, recv, count, n, rank_input, tmax, nch):
    """The ring's timed output against its own association (oracle fold_ring:
    chunk c of ring part k is folded along the ring from position c, the
    running partial as inout) on the first 4096 elements of every chunk of
    every part.  Max over ranks."""
    strides = M.ring_strides(n, nch)
    part = -(-(-(-count // len(strides))) // (n * 4)) * (n * 4)
    chunk = part // n
    xs = [rank_input(q, count) for q in range(n)]
    ok = True
    for k, st in enumerate(strides):
        for c in range(n):
            lo = min(k * part + c * chunk, count)
            hi = min(lo + 4096, min(k * part + part, count), lo + chunk)
            if hi <= lo:
                continue
            acc = xs[(c * st) % n][lo:hi].cpu().numpy()
            for i in range(1, n):
                acc = M.apply_op("SUM", "FLOAT", acc, xs[((c + i) * st) % n][lo:hi].cpu().numpy())
            ok &= bool(np.array_equal(recv[lo:hi].cpu().numpy().view(np.uint32), acc.view(np.uint32)))
    del xs
    (bad,) = tmax(0.0 if ok else 1.0)
    return bad == 0.0


def main():
    args = parse()
    n = int(os.environ.get("WORLD_SIZE", "1"))
    if n == 1:
        bench_local(args)
    else:
        bench_allreduce(args)


if __name__ == "__main__":
    main()
