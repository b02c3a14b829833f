"""Which fold_local_kernel<..., U> the host launches at 1 / 2 / 4 / 8 MiB per input (run under rocprofv3 --kernel-trace; the U is the last template argument)."""
import os, sys
sys.path.insert(0, "mpi.jl_amd")
import torch
import mpigx as MPI
os.environ.pop("MPIGX_LOCAL_U", None)
for mib in (1, 2, 4, 8):
    k = mib << 18
    xs = [torch.rand(k, device="cuda") for _ in range(8)]
    o = torch.empty(k, device="cuda")
    for _ in range(3):
        MPI.reduce_local_multi(xs, o, MPI.SUM)
    torch.cuda.synchronize()
    print(mib, "done", flush=True)
