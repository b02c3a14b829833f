"""mpigx — MI355X-native collective engine behind MPI.jl's collective API.

`import mpigx as MPI` gives the MPI.jl names (Init, COMM_WORLD, Comm_rank,
Allreduce_ (= Allreduce!), Reduce_, Bcast_, Allgather_, Alltoall_, Scan_,
Exscan_, SUM/MAX/..., Op, Datatype, Buffer, IN_PLACE, MPIError) over
libmpigx.so for device-resident (ROCm) buffers.
"""
from . import consts
from ._lib import DIAG_HEADER_PATH, HEADER_PATH, LIB_PATH, lib
from .api import *  # noqa: F401,F403
from .p2p import *  # noqa: F401,F403
from .rma import *  # noqa: F401,F403
from .types import Types  # noqa: F401
from .api import (IN_PLACE, Barrier, Buffer, Comm, Datatype, MPIError, Op, error_string,
                  reduce_local_multi)

# COMM_WORLD must not be a module attribute here: Init() rebinds
# api.COMM_WORLD, and __getattr__ below (consulted only for names the module
# does not have) hands out the live value, as MPI.COMM_WORLD is in MPI.jl
globals().pop("COMM_WORLD", None)


def free(obj):
    """MPI.free: communicators (comm.jl) and windows (onesided.jl:85-92)."""
    from . import api, rma
    if isinstance(obj, rma.Win):
        return rma.win_free(obj)
    return api.free(obj)


def __getattr__(name):
    # COMM_WORLD is rebound by Init(); expose the live value
    if name == "COMM_WORLD":
        from . import api
        return api.COMM_WORLD
    raise AttributeError(name)
