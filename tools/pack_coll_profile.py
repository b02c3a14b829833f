#!/usr/bin/env python3
"""Pack a tools/coll_prof.py summary (gpurun_out/coll_<tag>/<tag>_coll_summary.json)
into a compact profiles/ record: per config the device time, the all-rank HBM
fraction, rank 0's phase medians, the collective kernels' trace statistics and
the PMC traffic of rank 0's kernel against ONE rank's algorithmic bytes (the
counters cover the profiled process's own dispatches).

    python3 tools/pack_coll_profile.py <summary.json> <out.json>
"""
import json
import sys

# one rank's algorithmic HBM bytes per call, in units of the message S
# (tools/coll_prof.py algo_bytes / n at n = 2)
PER_RANK = {"pull": 2.5, "pull_generic": 2.5, "push": 3.0, "ring": 2.5, "pullpush": 2.0}


def short(k):
    return k.split("(")[0].replace("void ", "")


def main():
    s = json.load(open(sys.argv[1]))
    out = {"n": s["n"], "tag": s["tag"],
           "note": "ranks sharing one MI355X (same-device IPC); PMC traffic is rank 0's kernel only, compared with one "
                   "rank's algorithmic bytes; source: tools/coll_prof.py + tools/pack_coll_profile.py",
           "configs": {}}
    for cfg, v in s["configs"].items():
        mib, algo = cfg.split(":")
        algo = algo.split("/")[0]  # "pullpush/0": slice-count variant
        S = int(mib) << 20
        ph = v["run"].get("phases_us_per_rank")
        r = {"device_ms_median": v["run"]["device_ms_median"],
             "hbm_frac_of_8TBps_all_ranks": v["hbm_frac_of_8TBps"],
             "hbm_GBps_algorithmic_all_ranks": v["hbm_GBps_algorithmic"],
             "phases_us_rank0": ph[0] if ph else None,
             "kernels": {short(k): kv for k, kv in v["kernels"].items() if "mpigx" in k}}
        if v.get("traffic"):
            t = {}
            for k, kv in v["traffic"].items():
                if "mpigx" not in k or "copy_kernel" in k or "hbm_bytes_device" not in kv:
                    continue
                alg = PER_RANK[algo] * S
                t[short(k)] = {"FETCH_SIZE_KB": kv["FETCH_SIZE_KB_median"], "WRITE_SIZE_KB": kv["WRITE_SIZE_KB_median"],
                               "hbm_bytes_rank0": kv["hbm_bytes_device"], "algorithmic_bytes_per_rank": alg,
                               "traffic_over_algorithmic_per_rank": round(kv["hbm_bytes_device"] / alg, 4)}
            r["traffic"] = t
        out["configs"][cfg] = r
    json.dump(out, open(sys.argv[2], "w"), indent=1)


if __name__ == "__main__":
    main()
