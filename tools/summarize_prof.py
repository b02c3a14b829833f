"""Summarise rocprofv3 CSV output into profiles/<tag>_*.

kernel stats  -> profiles/<tag>_kernel_stats.csv   (copy of rocprofv3 --stats)
PMC traffic   -> profiles/<tag>_traffic.json       per-dispatch HBM bytes:
   bytes = 2 * FETCH_SIZE * 1024 + WRITE_SIZE * 1024
(gfx950: FETCH_SIZE reports half the bytes of a wide coalesced streaming read,
WRITE_SIZE is exact for 16-B streaming stores — MI355X_MICROARCH.md §HBM).
"""
import csv
import glob
import json
import os
import shutil
import statistics
import sys
from collections import defaultdict


def find(d, pat):
    return sorted(glob.glob(os.path.join(d, "**", pat), recursive=True))


def pmc_by_kernel(d, counter):
    vals = defaultdict(list)
    for f in find(d, "*counter_collection.csv"):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if row.get("Counter_Name") != counter:
                    continue
                vals[row.get("Kernel_Name", "?")].append(float(row["Counter_Value"]))
    return vals


def durations(d):
    res = defaultdict(list)
    for f in find(d, "*kernel_trace.csv"):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                res[row["Kernel_Name"]].append((int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) / 1e3)
    return res


def main(out, dest, tag):
    os.makedirs(dest, exist_ok=True)
    stats = find(os.path.join(out, "trace"), "*kernel_stats.csv")
    if stats:
        shutil.copy(stats[0], os.path.join(dest, f"{tag}_kernel_stats.csv"))
    fetch = pmc_by_kernel(os.path.join(out, "fetch"), "FETCH_SIZE")
    write = pmc_by_kernel(os.path.join(out, "write"), "WRITE_SIZE")
    dur = durations(os.path.join(out, "trace"))
    summary = {}
    for k in sorted(set(fetch) | set(write)):
        f = statistics.median(fetch[k]) if fetch.get(k) else None
        w = statistics.median(write[k]) if write.get(k) else None
        summary[k] = {"FETCH_SIZE_KB_median": f, "WRITE_SIZE_KB_median": w,
                      "hbm_bytes_per_dispatch": (2 * f * 1024 + w * 1024) if (f is not None and w is not None) else None,
                      "dispatches": len(fetch.get(k, [])),
                      "avg_us": statistics.mean(dur[k]) if dur.get(k) else None}
    # the headline kernel, keyed for bench.py
    j = {"kernels": summary}
    for k in summary:
        # the 256 MiB headline instantiation only (TREE, SH_FULL, U = 4): since
        # round 6 smaller inputs launch the U = 1 / 2 instantiations
        if "fold_local_kernel<mpigx::OpSum, float, 8, 0, 2, 4>" in k or "fold_local_kernelINS_5OpSumEfLi8ELi0ELi2ELi4E" in k:
            j["reduce_local_multi_f32_sum_8x256MiB"] = summary[k]["hbm_bytes_per_dispatch"]
    with open(os.path.join(dest, f"{tag}_traffic.json"), "w") as fh:
        json.dump(j, fh, indent=1)
    print(json.dumps({k: v for k, v in summary.items() if "mpigx" in k}, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:4])
