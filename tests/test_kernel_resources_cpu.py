"""Scratch (private segment) guard for the hot kernels, read from the built
gfx950 code objects' metadata — no GPU needed.

A kernel that lands in scratch runs an order of magnitude slower on a
one-vector-per-thread grid: the all-modes fold_kernel for float MAX copied
its 840-B FoldArgs to scratch per thread and ran config 2 at 0.67 TB/s
(DESIGN.md §5).  This pins the fix: every fold_local_kernel (config 2) has a
zero private segment, and so does every collective fold_kernel (float
MIN/MAX and NMAX-16 instantiations stage FoldArgs in LDS).
"""
import glob
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BUILD = os.path.join(ROOT, "mpi.jl_amd", "build")
LLVM = "/opt/rocm/lib/llvm/bin"


def _kernel_private_sizes(obj, tmp):
    fb, co = os.path.join(tmp, "fb.bin"), os.path.join(tmp, "co.elf")
    sec = subprocess.run([f"{LLVM}/llvm-readelf", "-S", obj], check=True, capture_output=True, text=True).stdout
    if ".hip_fatbin" not in sec:
        return {}  # a part without device kernels for this type (e.g. bitwise ops on bf16)
    subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fb}", obj, os.devnull], check=True)
    subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={fb}",
                    "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], check=True)
    notes = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", co], check=True,
                           capture_output=True, text=True).stdout
    sizes, name = {}, None
    for line in notes.splitlines():
        m = re.match(r"\s*\.name:\s+(\S+)", line)
        if m:
            name = m.group(1)
            continue
        m = re.match(r"\s*\.private_segment_fixed_size:\s+(\d+)", line)
        if m and name:
            sizes[name] = int(m.group(1))
    return sizes


# kern_rep.hip is built once per (type, op group): kern_<type>_p<part>.o
OBJS = sorted(glob.glob(os.path.join(BUILD, "kern_*_p*.o")))
REPS = sorted({re.sub(r"_p\d+\.o$", "", os.path.basename(o))[5:] for o in OBJS})


@pytest.mark.skipif(not OBJS or not os.path.exists(f"{LLVM}/clang-offload-bundler"),
                    reason="kernel objects not built (run __graft_entry__.build())")
@pytest.mark.parametrize("rep", REPS)
def test_hot_fold_kernels_have_no_scratch(rep, tmp_path):
    sizes = {}
    for obj in sorted(glob.glob(os.path.join(BUILD, f"kern_{rep}_p*.o"))):
        sizes.update(_kernel_private_sizes(obj, str(tmp_path)))
    local = {k: v for k, v in sizes.items() if "fold_local_kernel" in k}
    assert local, f"no fold_local_kernel for {rep}"
    assert all(v == 0 for v in local.values()), {k: v for k, v in local.items() if v}
    coll = {k: v for k, v in sizes.items() if "11fold_kernel" in k}
    assert coll, f"no fold_kernel for {rep}"
    assert all(v == 0 for v in coll.values()), {k: v for k, v in coll.items() if v}
    # ring reduce-scatter + allgather, Scan / Exscan and the dedicated
    # zero-copy two-shot (ar_zc_kernel, U vectors per thread) likewise
    zc = {k: v for k, v in sizes.items() if "12ar_zc_kernel" in k}
    assert len(zc) >= 5, f"ar_zc_kernel instantiations missing for {rep}"
    other = {k: v for k, v in sizes.items() if "11ring_kernel" in k or "11scan_kernel" in k or "12ar_zc_kernel" in k}
    assert other, f"no ring/scan kernel for {rep}"
    assert all(v == 0 for v in other.values()), {k: v for k, v in other.items() if v}
