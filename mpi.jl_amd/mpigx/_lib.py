"""ctypes binding of libmpigx.so (include/mpigx.h + include/mpigx_diag.h).

The library is built in-tree (mpi.jl_amd/lib/libmpigx.so, see
mpi.jl_amd/csrc/Makefile).  There is no fallback: if the shared object is
missing, loading fails loudly.
"""
from __future__ import annotations

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("MPIGX_LIB", os.path.join(os.path.dirname(_HERE), "lib", "libmpigx.so"))
HEADER_PATH = os.path.join(os.path.dirname(os.path.dirname(_HERE)), "include", "mpigx.h")
# diagnostic exports (phase stamps, slot / mapping checks, tuner statistics,
# probes): not part of the MPI-facing ABI
DIAG_HEADER_PATH = os.path.join(os.path.dirname(os.path.dirname(_HERE)), "include", "mpigx_diag.h")

_lib = None

c_int, c_void_p, c_longlong, c_size_t = ctypes.c_int, ctypes.c_void_p, ctypes.c_longlong, ctypes.c_size_t


_IP = ctypes.POINTER(ctypes.c_int)


class UniqueId(ctypes.Structure):
    _fields_ = [("internal", ctypes.c_char * 128)]


USER_FN = ctypes.CFUNCTYPE(None, c_void_p, c_void_p, ctypes.POINTER(c_int), ctypes.POINTER(c_int))
DEVICE_FN = ctypes.CFUNCTYPE(None, c_void_p, c_void_p, c_longlong, c_int, c_void_p)

# name -> (restype, argtypes)
PROTOTYPES = {
    "mpigx_get_version": (c_int, [ctypes.POINTER(c_int), ctypes.POINTER(c_int)]),
    "mpigx_error_string": (c_int, [c_int, ctypes.c_char_p, ctypes.POINTER(c_int)]),
    "mpigx_query_thread": (c_int, [ctypes.POINTER(c_int)]),
    "mpigx_op_valid": (c_int, [c_int, c_int]),
    "mpigx_type_size": (c_int, [c_int, ctypes.POINTER(c_int)]),
    "mpigx_get_unique_id": (c_int, [ctypes.POINTER(UniqueId)]),
    "mpigx_comm_init_rank": (c_int, [ctypes.POINTER(c_void_p), c_int, ctypes.POINTER(UniqueId), c_int, c_int]),
    "mpigx_comm_free": (c_int, [c_void_p]),
    "mpigx_comm_split": (c_int, [c_void_p, c_int, c_int, ctypes.POINTER(c_void_p)]),
    "mpigx_comm_rank": (c_int, [c_void_p, ctypes.POINTER(c_int)]),
    "mpigx_comm_size": (c_int, [c_void_p, ctypes.POINTER(c_int)]),
    "mpigx_comm_device": (c_int, [c_void_p, ctypes.POINTER(c_int)]),
    "mpigx_comm_set_stream": (c_int, [c_void_p, c_void_p]),
    "mpigx_comm_set_blocking": (c_int, [c_void_p, c_int]),
    "mpigx_comm_synchronize": (c_int, [c_void_p]),
    "mpigx_comm_set_reduce_order": (c_int, [c_void_p, c_int]),
    "mpigx_comm_set_knob": (c_int, [c_void_p, c_int, c_longlong]),
    "mpigx_comm_get_knob": (c_int, [c_void_p, c_int, ctypes.POINTER(c_longlong)]),
    "mpigx_comm_device_share": (c_int, [c_void_p, ctypes.POINTER(c_int), ctypes.POINTER(c_int)]),
    "mpigx_comm_set_stamps": (c_int, [c_void_p, c_void_p]),
    "mpigx_comm_set_timeout": (c_int, [c_void_p, c_longlong]),
    "mpigx_comm_release": (c_int, [c_void_p]),
    "mpigx_comm_diag_slots": (c_int, [c_void_p, c_int, c_void_p, c_void_p]),
    "mpigx_comm_diag_mapcheck": (c_int, [c_void_p, ctypes.c_ulonglong, c_void_p]),
    "mpigx_comm_diag_state": (c_int, [c_void_p, c_void_p]),
    "mpigx_comm_diag_break": (c_int, [c_void_p]),
    "mpigx_comm_diag_peer_mem": (c_int, [c_void_p, ctypes.POINTER(ctypes.c_uint), ctypes.POINTER(ctypes.c_uint)]),
    "mpigx_comm_zc_stats": (c_int, [c_void_p, ctypes.POINTER(ctypes.c_ulonglong), ctypes.POINTER(ctypes.c_ulonglong)]),
    "mpigx_comm_host_stats": (c_int, [c_void_p, ctypes.POINTER(ctypes.c_double)]),
    "mpigx_comm_ar_choice": (c_int, [c_void_p, ctypes.POINTER(c_int), ctypes.POINTER(ctypes.c_double),
                                     ctypes.POINTER(ctypes.c_double)]),
    "mpigx_comm_ar_costs": (c_int, [c_void_p, ctypes.POINTER(c_int), ctypes.POINTER(ctypes.c_double)]),
    "mpigx_comm_tune_class": (c_int, [c_void_p, c_int, ctypes.POINTER(c_int), ctypes.POINTER(ctypes.c_double)]),
    "mpigx_comm_probe": (c_int, [c_void_p, c_int, c_longlong, ctypes.POINTER(ctypes.c_double)]),
    "mpigx_read_probe": (c_int, [ctypes.POINTER(c_void_p), c_int, c_longlong, c_void_p, c_void_p]),
    "mpigx_mix_probe": (c_int, [ctypes.POINTER(c_void_p), c_int, c_longlong, c_void_p, c_void_p]),
    "mpigx_barrier": (c_int, [c_void_p]),
    "mpigx_bcast": (c_int, [c_void_p, c_int, c_int, c_int, c_void_p]),
    "mpigx_allgather": (c_int, [c_void_p, c_int, c_int, c_void_p, c_int, c_int, c_void_p]),
    "mpigx_alltoall": (c_int, [c_void_p, c_int, c_int, c_void_p, c_int, c_int, c_void_p]),
    "mpigx_gather": (c_int, [c_void_p, c_int, c_int, c_void_p, c_int, c_int, c_int, c_void_p]),
    "mpigx_gatherv": (c_int, [c_void_p, c_int, c_int, c_void_p, _IP, _IP, c_int, c_int, c_void_p]),
    "mpigx_scatter": (c_int, [c_void_p, c_int, c_int, c_void_p, c_int, c_int, c_int, c_void_p]),
    "mpigx_scatterv": (c_int, [c_void_p, _IP, _IP, c_int, c_void_p, c_int, c_int, c_int, c_void_p]),
    "mpigx_allgatherv": (c_int, [c_void_p, c_int, c_int, c_void_p, _IP, _IP, c_int, c_void_p]),
    "mpigx_alltoallv": (c_int, [c_void_p, _IP, _IP, c_int, c_void_p, _IP, _IP, c_int, c_void_p]),
    "mpigx_reduce": (c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_void_p]),
    "mpigx_allreduce": (c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_void_p]),
    "mpigx_scan": (c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_void_p]),
    "mpigx_exscan": (c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_void_p]),
    "mpigx_reduce_local": (c_int, [c_void_p, c_void_p, c_int, c_int, c_int]),
    "mpigx_reduce_local_multi": (c_int, [ctypes.POINTER(c_void_p), c_int, c_void_p, c_longlong, c_int, c_int, c_int,
                                         c_void_p]),
    # point-to-point
    "mpigx_send": (c_int, [c_void_p, c_int, c_int, c_int, c_int, c_void_p]),
    "mpigx_isend": (c_int, [c_void_p, c_int, c_int, c_int, c_int, c_void_p, _IP]),
    "mpigx_recv": (c_int, [c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_void_p]),
    "mpigx_irecv": (c_int, [c_void_p, c_int, c_int, c_int, c_int, c_void_p, _IP]),
    "mpigx_sendrecv": (c_int, [c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_int, c_int, c_int, c_int,
                               c_void_p, c_void_p]),
    "mpigx_probe": (c_int, [c_int, c_int, c_void_p, c_void_p]),
    "mpigx_iprobe": (c_int, [c_int, c_int, c_void_p, _IP, c_void_p]),
    "mpigx_get_count": (c_int, [c_void_p, c_int, _IP]),
    "mpigx_test_cancelled": (c_int, [c_void_p, _IP]),
    "mpigx_wait": (c_int, [_IP, c_void_p]),
    "mpigx_test": (c_int, [_IP, _IP, c_void_p]),
    "mpigx_waitall": (c_int, [c_int, _IP, c_void_p]),
    "mpigx_testall": (c_int, [c_int, _IP, _IP, c_void_p]),
    "mpigx_waitany": (c_int, [c_int, _IP, _IP, c_void_p]),
    "mpigx_testany": (c_int, [c_int, _IP, _IP, _IP, c_void_p]),
    "mpigx_waitsome": (c_int, [c_int, _IP, _IP, _IP, c_void_p]),
    "mpigx_testsome": (c_int, [c_int, _IP, _IP, _IP, c_void_p]),
    "mpigx_cancel": (c_int, [_IP]),
    "mpigx_request_free": (c_int, [_IP]),
    # one-sided
    "mpigx_win_create": (c_int, [c_void_p, c_longlong, c_int, c_void_p, ctypes.POINTER(c_void_p)]),
    "mpigx_win_create_dynamic": (c_int, [c_void_p, ctypes.POINTER(c_void_p)]),
    "mpigx_win_allocate_shared": (c_int, [c_longlong, c_int, c_void_p, c_void_p, ctypes.POINTER(c_void_p)]),
    "mpigx_win_shared_query": (c_int, [c_void_p, c_int, ctypes.POINTER(c_longlong), _IP, c_void_p]),
    "mpigx_win_free": (c_int, [ctypes.POINTER(c_void_p)]),
    "mpigx_win_attach": (c_int, [c_void_p, c_void_p, c_longlong]),
    "mpigx_win_detach": (c_int, [c_void_p, c_void_p]),
    "mpigx_win_fence": (c_int, [c_int, c_void_p]),
    "mpigx_win_flush": (c_int, [c_int, c_void_p]),
    "mpigx_win_sync": (c_int, [c_void_p]),
    "mpigx_win_lock": (c_int, [c_int, c_int, c_int, c_void_p]),
    "mpigx_win_unlock": (c_int, [c_int, c_void_p]),
    "mpigx_win_get_flavor": (c_int, [c_void_p, _IP]),
    "mpigx_get": (c_int, [c_void_p, c_int, c_int, c_int, c_longlong, c_int, c_int, c_void_p]),
    "mpigx_put": (c_int, [c_void_p, c_int, c_int, c_int, c_longlong, c_int, c_int, c_void_p]),
    "mpigx_fetch_and_op": (c_int, [c_void_p, c_void_p, c_int, c_int, c_longlong, c_int, c_void_p]),
    "mpigx_accumulate": (c_int, [c_void_p, c_int, c_int, c_int, c_longlong, c_int, c_int, c_int, c_void_p]),
    "mpigx_get_accumulate": (c_int, [c_void_p, c_int, c_int, c_void_p, c_int, c_int, c_int, c_longlong, c_int, c_int,
                                     c_int, c_void_p]),
    # derived datatypes
    "mpigx_type_contiguous": (c_int, [c_int, c_int, _IP]),
    "mpigx_type_vector": (c_int, [c_int, c_int, c_int, c_int, _IP]),
    "mpigx_type_create_hvector": (c_int, [c_int, c_int, c_longlong, c_int, _IP]),
    "mpigx_type_create_subarray": (c_int, [c_int, _IP, _IP, _IP, c_int, c_int, _IP]),
    "mpigx_type_create_struct": (c_int, [c_int, _IP, ctypes.POINTER(c_longlong), _IP, _IP]),
    "mpigx_type_create_resized": (c_int, [c_int, c_longlong, c_longlong, _IP]),
    "mpigx_type_commit": (c_int, [_IP]),
    "mpigx_type_free": (c_int, [_IP]),
    "mpigx_type_get_extent": (c_int, [c_int, ctypes.POINTER(c_longlong), ctypes.POINTER(c_longlong)]),
    "mpigx_type_get_true_extent": (c_int, [c_int, ctypes.POINTER(c_longlong), ctypes.POINTER(c_longlong)]),
    "mpigx_type_size_x": (c_int, [c_int, ctypes.POINTER(c_longlong)]),
    "mpigx_pack_size": (c_int, [c_int, c_int, ctypes.POINTER(c_longlong)]),
    "mpigx_pack": (c_int, [c_void_p, c_int, c_int, c_void_p, c_longlong, ctypes.POINTER(c_longlong), c_void_p]),
    "mpigx_unpack": (c_int, [c_void_p, c_longlong, ctypes.POINTER(c_longlong), c_void_p, c_int, c_int, c_void_p]),
    # user-defined ops
    "mpigx_op_create": (c_int, [USER_FN, c_int, _IP]),
    "mpigx_op_create_device": (c_int, [DEVICE_FN, c_int, _IP]),
    "mpigx_op_free": (c_int, [_IP]),
    "mpigx_op_commutative": (c_int, [c_int, _IP]),
    "mpigx_malloc": (c_int, [ctypes.POINTER(c_void_p), c_size_t]),
    "mpigx_free": (c_int, [c_void_p]),
    "mpigx_memcpy": (c_int, [c_void_p, c_void_p, c_size_t]),
}


def lib():
    """Load libmpigx.so (once).  Raises if the HIP extension was not built."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(
                f"libmpigx.so not found at {LIB_PATH}: build it with `make -C mpi.jl_amd/csrc` "
                "(or __graft_entry__.build()); mpigx has no CPU fallback")
        L = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
        for name, (res, args) in PROTOTYPES.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib
