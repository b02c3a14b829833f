"""Derived datatypes exercised by the pack / unpack parity checks: the shapes
MPI.jl builds (buffers.jl:104-117 vector / subarray views, datatypes.jl:269-316
isbits structs and primitive types, test/test_datatype.jl's Boundary,
Boundary2, Primitive16/24/80, NTuple{3,UInt8}, Nothing) plus the Types
constructors (contiguous, vector, hvector, subarray C/Fortran, struct with
out-of-order displacements, resized, nesting)."""
import numpy as np

BOUNDARY = np.dtype([("c", np.uint16), ("a", np.int64), ("b", np.uint8)], align=True)
BOUNDARY2 = np.dtype([("a", np.uint32), ("b", np.dtype([("f0", np.int64), ("f1", np.uint8)], align=True)),
                      ("c", np.dtype([]))], align=True)
NTUPLE3 = np.dtype([("f0", np.uint8), ("f1", np.uint8), ("f2", np.uint8)])


def build(MPI):
    """[(name, Datatype)] — all committed."""
    T = MPI.Types
    D = MPI.Datatype
    i16, i32, i64, f32, f64 = (D(np.int16), D(np.int32), D(np.int64), D(np.float32), D(np.float64))
    c = T.commit_
    out = [
        ("vector_3_2_5_i64", c(T.create_vector(3, 2, 5, i64))),
        ("vector_col_f64", c(T.create_vector(4, 1, 4, f64))),
        ("subarray_C_f32", c(T.create_subarray([4, 5], [2, 3], [1, 1], f32, rowmajor=True))),
        ("subarray_F_f32", c(T.create_subarray([4, 5], [2, 3], [1, 1], f32))),
        ("subarray_3d_i16", c(T.create_subarray([3, 4, 5], [2, 2, 3], [1, 0, 2], i16, rowmajor=True))),
        ("hvector_3_2_20_i16", c(T.create_hvector(3, 2, 20, i16))),
        ("contig_2_vector", c(T.create_contiguous(2, T.create_vector(2, 1, 3, i32)))),
        ("resized_vector", c(T.create_resized(T.create_vector(2, 1, 3, i32), 0, 8))),
        ("struct_out_of_order", c(T.create_struct([1, 2], [16, 0], [f64, i32]))),
        ("boundary", D(BOUNDARY)),
        ("boundary2", D(BOUNDARY2)),
        ("primitive16", D(np.dtype("V2"))),
        ("primitive24", D(np.dtype("V3"))),
        ("primitive80", D(np.dtype("V10"))),
        ("ntuple3", D(NTUPLE3)),
        ("nothing", D(np.dtype([]))),
        ("vector_of_struct", c(T.create_vector(2, 1, 2, D(BOUNDARY)))),
        ("contig_3_boundary", c(T.create_contiguous(3, D(BOUNDARY)))),
    ]
    return out


def typed_input(extent, true_ub, count):
    n = max(1, extent * count + max(0, true_ub) + 64)
    return ((np.arange(n, dtype=np.int64) * 7 + 3) % 251).astype(np.uint8)
