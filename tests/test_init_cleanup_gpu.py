"""A communicator rendezvous that times out (a peer never arrives) leaves
nothing behind: no /dev/shm/mpigx-* segment, no device allocation
(mpigx.cpp comm_init / comm_release)."""
import ctypes
import os

import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu


def test_init_timeout_leaks_nothing():
    """(~1 s) A communicator init that times out releases every resource it took (device memory, pinned page, shm name)."""
    import mpigx
    from mpigx._lib import UniqueId
    L = mpigx.lib()
    os.environ["MPIGX_INIT_TIMEOUT_MS"] = "300"
    os.environ["MPIGX_STAGING_BYTES"] = str(1 << 30)  # large enough to see in mem_get_info
    try:
        torch.cuda.init()
        torch.cuda.synchronize()
        free0, _ = torch.cuda.mem_get_info(0)
        for rank in (0, 1):  # rank 0 creates the shm block; rank 1 waits for one that never appears
            uid = UniqueId()
            assert L.mpigx_get_unique_id(ctypes.byref(uid)) == 0
            name = ctypes.string_at(ctypes.addressof(uid), 64).split(b"\0")[0].decode()
            comm = ctypes.c_void_p()
            rc = L.mpigx_comm_init_rank(ctypes.byref(comm), 2, ctypes.byref(uid), rank, 0)
            assert rc == 15, rc  # MPI_ERR_OTHER: the peer did not arrive
            assert not comm.value
            assert not os.path.exists("/dev/shm" + name), name
            leftovers = [f for f in os.listdir("/dev/shm") if f.startswith(f"mpigx-{os.getpid()}-")]
            assert not leftovers, leftovers
        free1, _ = torch.cuda.mem_get_info(0)
        assert free0 - free1 < (256 << 20), (free0, free1)
    finally:
        os.environ.pop("MPIGX_INIT_TIMEOUT_MS", None)
        os.environ.pop("MPIGX_STAGING_BYTES", None)
