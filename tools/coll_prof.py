#!/usr/bin/env python3
"""rocprofv3 profiles of the collective kernels (VERDICT r02 "R3"): every rank
runs as its own `rocprofv3 ... -- python3 tools/coll_rank.py`, started by this
parent, which never touches the GPU (no torch import here), so no profiled
process is exec'ed from one that initialised it.

    python3 tools/coll_prof.py <out_dir> <tag> [--n 2] [--configs 256:pull,16:pull,...]

Per config (MiB:algo) three passes, each a fresh set of rank processes:
  trace : every rank under `rocprofv3 --kernel-trace --stats` -> kernel stats;
  fetch : rank 0 under `rocprofv3 --pmc FETCH_SIZE --kernel-trace`, the other
          ranks unprofiled;
  write : the same with WRITE_SIZE (FETCH_SIZE and WRITE_SIZE do not fit one
          TCC pass).
Measured (r03): the counters cover the profiled process's own dispatches
only (rank 0's kernel: 2.50 S for a pull two-shot of S bytes at n = 2, which
is one rank's algorithmic traffic), so traffic is compared with ONE rank's
algorithmic bytes (all-rank bytes / n).  gfx950: FETCH_SIZE reports half the bytes of a 16-B/lane
streaming read (MI355X_MICROARCH.md §HBM), so bytes = 2 * FETCH + WRITE.
Writes <out_dir>/<config>_<pass>/..., and <out_dir>/<tag>_coll_summary.json.
"""
import argparse
import csv
import glob
import json
import os
import socket
import statistics
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KERNEL_KEYS = ("ar_zc_kernel", "fold_kernel", "ring_kernel", "copy_kernel")


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def run_ranks(n, mib, algo, prof, outdir, iters, timeout, slices=None):
    """prof(rank) -> rocprofv3 argument list (or None).  Returns rank 0's JSON."""
    port = free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(n), LOCAL_RANK=str(r), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), TMPDIR="/tmp", MPIGX_DEVICE="0", MPIGX_TIMEOUT_MS="20000")
        cmd = [sys.executable, os.path.join(ROOT, "tools", "coll_rank.py"), "--mib", str(mib), "--algo", algo,
               "--iters", str(iters)] + ([] if slices is None else ["--slices", str(slices)])
        p = prof(r)
        if p:
            cmd = ["rocprofv3", *p, "-d", os.path.join(outdir, f"rank{r}"), "-o", "run", "--output-format", "csv",
                   "--", *cmd]
        log = open(os.path.join(outdir, f"rank{r}.log"), "w")
        procs.append((subprocess.Popen(["timeout", "-k", "10", str(timeout), *cmd], env=env, cwd="/tmp",
                                       stdout=log, stderr=subprocess.STDOUT), log))
    rcs = []
    for p, log in procs:
        rcs.append(p.wait())
        log.close()
    if any(rcs):
        raise RuntimeError(f"ranks exited {rcs} ({outdir})")
    for line in open(os.path.join(outdir, "rank0.log")):
        if line.startswith("{"):
            return json.loads(line)
    raise RuntimeError(f"no result line ({outdir})")


def kernel_rows(d):
    """{kernel name: [durations us]} of the collective kernels in a trace dir."""
    res = {}
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                k = row["Kernel_Name"]
                if any(x in k for x in KERNEL_KEYS):
                    res.setdefault(k, []).append((int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) / 1e3)
    return res


def pmc(d, counter):
    res = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if row.get("Counter_Name") == counter and any(x in row.get("Kernel_Name", "") for x in KERNEL_KEYS):
                    res.setdefault(row["Kernel_Name"], []).append(float(row["Counter_Value"]))
    return res


def algo_bytes(algo, n, S):
    """Algorithmic HBM bytes of one call, all n ranks together (same device).
    pull / ring: per rank RS reads n chunks of S/n and writes S/n, AG reads and
    writes (n-1)S/n -> S(2 + (n-1)/n).  push: per rank phase 1 reads and writes
    (n-1)S/n (peers' arena slots), phase 2 reads S (slots + own chunk) and
    writes S (own + peers' recvbufs) -> 2S(1 + (n-1)/n).  pullpush: per rank
    the fold reads n chunks of S/n and writes its chunk into n recvbufs -> 2S."""
    if algo.startswith("pullpush"):
        return n * 2 * S
    if algo == "push":
        return n * 2 * S * (1 + (n - 1) / n)
    return n * S * (2 + (n - 1) / n)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("out")
    ap.add_argument("tag")
    ap.add_argument("--n", type=int, default=2)
    ap.add_argument("--configs", default="256:pull,256:pullpush,256:pull_generic,256:push,256:ring,16:pull,16:pullpush")
    ap.add_argument("--pmc-configs", default="256:pull,256:pullpush,16:pull")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--timeout", type=int, default=150)
    a = ap.parse_args()
    a.out = os.path.abspath(a.out)  # the ranks (and rocprofv3's -d) run with cwd /tmp
    os.makedirs(a.out, exist_ok=True)
    summary = {"n": a.n, "tag": a.tag, "configs": {}}
    pmc_set = set(a.pmc_configs.split(",")) if a.pmc_configs else set()
    for cfg in a.configs.split(","):
        mib, algo = cfg.split(":")
        mib = int(mib)
        slices = None
        if "/" in algo:  # "pullpush/0": with MPIGX_AR_SLICES = 0
            algo, sl = algo.split("/")
            slices = int(sl)
        tag = algo if slices is None else f"{algo}_s{slices}"
        S = mib << 20
        rec = {}
        d = os.path.join(a.out, f"{mib}MiB_{tag}_trace")
        os.makedirs(d, exist_ok=True)
        res = run_ranks(a.n, mib, algo, lambda r: ["--kernel-trace", "--stats"], d, a.iters, a.timeout, slices)
        rec["run"] = res
        rows = kernel_rows(d)
        rec["kernels"] = {k: {"dispatches": len(v), "avg_us": round(statistics.mean(v), 2),
                              "median_us": round(statistics.median(v), 2)} for k, v in rows.items()}
        for f in glob.glob(os.path.join(d, "rank0", "**", "*kernel_stats.csv"), recursive=True):
            rec["kernel_stats_csv"] = os.path.relpath(f, a.out)
        if cfg in pmc_set:
            tr = {}
            for counter in ("FETCH_SIZE", "WRITE_SIZE"):
                dp = os.path.join(a.out, f"{mib}MiB_{tag}_{counter.lower()}")
                os.makedirs(dp, exist_ok=True)
                run_ranks(a.n, mib, algo, lambda r, c=counter: ["--pmc", c, "--kernel-trace"] if r == 0 else None,
                          dp, 5, a.timeout, slices)
                for k, v in pmc(dp, counter).items():
                    tr.setdefault(k, {})[counter + "_KB_median"] = statistics.median(v)
            for k, v in tr.items():
                if "FETCH_SIZE_KB_median" in v and "WRITE_SIZE_KB_median" in v:
                    b = 2 * v["FETCH_SIZE_KB_median"] * 1024 + v["WRITE_SIZE_KB_median"] * 1024
                    v["hbm_bytes_device"] = b
                    v["algorithmic_bytes_all_ranks"] = algo_bytes(algo, a.n, S)
                    v["traffic_over_algorithmic_per_rank"] = round(b * a.n / algo_bytes(algo, a.n, S), 4)
            rec["traffic"] = tr
        dev_s = res["device_ms_median"] / 1e3
        rec["hbm_GBps_algorithmic"] = round(algo_bytes(algo, a.n, S) / dev_s / 1e9, 1)
        rec["hbm_frac_of_8TBps"] = round(algo_bytes(algo, a.n, S) / dev_s / 8e12, 4)
        summary["configs"][cfg] = rec
        print(json.dumps({cfg: {"device_ms": res["device_ms_median"], "hbm_frac": rec["hbm_frac_of_8TBps"],
                                "phases_rank0": res["phases_us_per_rank"][0]}}), flush=True)
    with open(os.path.join(a.out, f"{a.tag}_coll_summary.json"), "w") as fh:
        json.dump(summary, fh, indent=1)


if __name__ == "__main__":
    main()
