"""bench.py's two JSON line shapes, built on the CPU from recorded section
outputs: the N = 1 line (config 2, BENCH_r05's numbers)
and the N > 1 line (config 3, the N = 2 run recorded in
profiles/r05zq_bench_n2_1gpu_xdev.json).  Both must carry a non-null
roofline, cpu_baseline and config.workload; the N > 1 line's cpu_baseline is
the same-run MPICH 8-rank MPI_Allreduce (the reference path behind
/root/reference/src/collective.jl:698-700), and its same-device roofline
quotes the newest collective PMC profile, whatever its suffix."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402

REC_N2 = os.path.join(ROOT, "profiles", "r05zq_bench_n2_1gpu_xdev.json")


def _required(line):
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "dtype", "data", "config", "roofline", "cpu_baseline"):
        assert k in line, k
    assert line["config"].get("workload"), line["config"]
    r = line["roofline"]
    assert r is not None and all(r.get(k) is not None for k in ("bound", "achieved", "peak", "unit", "frac")), r
    assert abs(r["frac"] - r["achieved"] / r["peak"]) < 1e-3
    cb = line["cpu_baseline"]
    assert cb is not None and all(cb.get(k) is not None for k in ("value", "unit", "cores", "kind", "sample")), cb
    assert cb["kind"] in ("reference", "port")
    json.dumps(line)  # one JSON line


def test_local_line_shape():
    m = {"nbuf": 8, "mib": 256, "steps": 20, "warmup": 5, "wall_s": 0.3833e-3, "kern_ms": 0.3823,
         "read_ms": [0.3050, 0.3061], "mix_ms": [0.3760, 0.3771], "parity": True,
         "variants": {"f32_MAX_GBps": 6500.0}, "sweep": {"1MiB": {"GBps": 1400.0, "us": 6.74}},
         "cpu": {"value": 24.66, "unit": "GB/s", "cores": 1, "kind": "reference",
                 "sample": "MPICH 3.3.2 MPI_Reduce_local, 8 x 256 MiB f32 SUM", "sec_per_step": 0.098},
         "cpu_ar": None, "traffic": 2415988736.0, "traffic_src": "profiles/r05zt_traffic.json"}
    line = bench.build_local_line(m)
    _required(line)
    assert line["n_gpus"] == 1 and line["roofline"]["bound"] == "hbm"
    assert abs(line["value"] - 2415919104 / 0.3833e-3 / 1e9) < 0.01
    r = line["roofline"]
    # peak_measured is the fold's own 8 : 1 mix, the read-only stream beside it
    assert abs(r["peak_measured"] - 2415919104 / 0.3760e-3 / 1e9) < 0.1
    assert abs(r["peak_read_only"] - 8 * (256 << 20) / 0.3050e-3 / 1e9) < 0.1
    assert r["frac_vs_measured"] is not None and r["frac_vs_read_only"] is not None


def test_coll_line_shape_from_recorded_run():
    rec = json.load(open(REC_N2))
    n = rec["n_gpus"]
    t = rec["ms_per_step"] / 1e3
    kern = (256 << 20) / (rec["roofline"]["busbw_device_GBps"] * 1e9) * 2 * (n - 1) / n
    kind = "pullpush"
    traffic, src = bench.coll_traffic_from_profiles(kind, n, 256)
    m = {"n": n, "mib": 256, "steps": rec["steps"], "warmup": rec["warmup"], "t": t, "kern": kern,
         "same_device": True, "ar_tune": rec["ar_tune"], "traffic": traffic, "traffic_src": src,
         "xg": rec["roofline"]["xgmi_traffic"], "cpu_ar": rec["cpu_reference_allreduce"], "correct": rec["correct"],
         "tune_classes": rec["tune_classes"], "probe": rec["xgmi_probe_informational"],
         "phases": rec["phases_headline_us"], "section_s": rec["section_wall_s"], "sweep": rec["sweep_mpigx_busbw"],
         "rccl": rec["rccl_busbw"], "cfg4": rec["config4_bcast_allgather_alltoall"],
         "tune_classes4": rec["tune_classes_after_config4"], "cfg5": rec["config5_scan_exscan_reduce"]["cases"],
         "cfg5_ok": rec["config5_scan_exscan_reduce"]["bit_exact_all"], "errors": rec["errors"]}
    line = bench.build_coll_line(m)
    _required(line)
    assert abs(line["value"] - rec["value"]) < 0.5
    cb = line["cpu_baseline"]
    assert cb["kind"] == "reference" and cb["cores"] == 8 and cb["value"] == round(rec["cpu_reference_allreduce"]
                                                                                  ["busbw_GBps"], 3)
    assert "MPI_Allreduce" in cb["sample"] and cb["model"]
    # the newest collective PMC profile, whatever its suffix (r05zh_..._xdev_fullgrid)
    assert src is not None and "r05zh" in src, src
    assert line["roofline"]["traffic"] == traffic


def test_coll_line_on_distinct_gpus_and_failed_baseline():
    """The driver's 8-GPU shape: bound xgmi; and a baseline run that failed
    gives cpu_baseline None (reported, not invented)."""
    m = {"n": 8, "mib": 256, "steps": 20, "warmup": 5, "t": 1.0e-3, "kern": 0.9e-3, "same_device": False,
         "ar_tune": {"choice": "pull two-shot"}, "traffic": None, "traffic_src": None, "xg": None,
         "cpu_ar": {"ranks": 8, "cores": 8, "mib": 256, "iters": 3, "sec_per_call": 0.27, "algbw_GBps": 0.99,
                    "busbw_GBps": 1.73, "model": "AMD EPYC"},
         "correct": {"sample_bit_exact_vs_oracle": True}, "tune_classes": {}, "probe": {}, "phases": {},
         "section_s": {}, "sweep": {}, "rccl": {}, "cfg4": {}, "tune_classes4": {}, "cfg5": {}, "cfg5_ok": True,
         "errors": {}}
    line = bench.build_coll_line(m)
    _required(line)
    assert line["roofline"]["bound"] == "xgmi" and line["roofline"]["peak"] == round(7 * bench.XGMI_LINK_GBPS, 1)
    assert line["cpu_baseline"]["value"] == 1.73
    m["cpu_ar"] = {"error": "timeout"}
    assert bench.build_coll_line(m)["cpu_baseline"] is None


def test_cpu_reference_sweep_runs_here():
    """The N > 1 line's reference sweep (oracle/mpich_bench.c `sweep`, MPICH
    under mpiexec) at a small size here: every section present, positive
    rates.  Skipped where MPICH is absent."""
    import pytest
    exe = os.path.join(ROOT, "oracle", "_ref", "mpich_bench")
    if not (os.path.exists(exe) and os.path.exists("/opt/conda/bin/mpiexec")):
        pytest.skip("MPICH harness not built here")
    j = bench.cpu_reference_sweep(ranks=2, maxmib=1)
    assert "error" not in j, j
    assert j["ranks"] == 2 and j["kind"] == "reference"
    assert j["allreduce_8KiB"]["busbw_GBps"] > 0 and j["allreduce_1024KiB"]["algbw_GBps"] > 0
    assert j["movers_64KiB"]["alltoall_busbw_GBps"] > 0 and j["movers_1024KiB"]["bcast_busbw_GBps"] > 0
    for d in ("int32", "int64"):
        for o in ("BAND", "BOR", "MAX"):
            assert j[f"{d}_{o}_1024"]["scan_algbw_GBps"] > 0
