"""CPU (gloo) rank process: the unique-id bootstrap of mpigx.Init's N>1 path.
Prints the id every rank ended up with; no GPU is touched."""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "mpi.jl_amd"))

import ctypes  # noqa: E402

from mpigx import api  # noqa: E402

rank, size = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
uid = api._bootstrap_id(rank, size)
raw = ctypes.string_at(ctypes.addressof(uid), 128)
import torch.distributed as dist  # noqa: E402

objs = [None] * size
dist.all_gather_object(objs, raw.hex())
assert len(set(objs)) == 1, objs
assert raw.startswith(b"/mpigx-") and raw[64:72] == b"60vxgipm"
print("BOOT", rank, raw[:40].decode(errors="replace").rstrip("\x00"), flush=True)
dist.destroy_process_group()
