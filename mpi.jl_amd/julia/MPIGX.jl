# MPIGX.jl — the MPI.jl side of the drop-in: device-resident buffers go to
# libmpigx.so (MI355X engine) through ccall; everything else keeps going to
# libmpi exactly as before.
#
# Load after MPI.jl:   using MPI; include("mpi.jl_amd/julia/MPIGX.jl"); using .MPIGX
#
# Plug points used (the only extension hooks MPI.jl offers, SURVEY.md §8b):
#   * a device buffer type + Base.cconvert/unsafe_convert(::Type{MPIPtr}, ...)
#     (src/buffers.jl:13-23, the role src/cuda.jl:6-24 plays for CuArray);
#   * Datatype(T) for BFloat16 (src/datatypes.jl:269-292);
#   * multiple dispatch on the collective signatures of src/collective.jl —
#     the methods below have the reference's argument lists and differ only in
#     the ccall target (:mpigx_* in libmpigx instead of :MPI_* in libmpi).
# Julia is not installed in the build image, so this file is untested here;
# the Python mirror (mpi.jl_amd/mpigx) exercises the same C ABI.
module MPIGX

using MPI
import MPI: Comm, Op, Datatype, MPIPtr, SentinelPtr, MPI_Op, MPI_Datatype, @mpichk,
            Allreduce!, Reduce!, Bcast!, Allgather!, Alltoall!, Scan!, Exscan!

const libmpigx = get(ENV, "MPIGX_LIB", joinpath(@__DIR__, "..", "lib", "libmpigx.so"))
const MPIGX_BFLOAT16 = Cint(1275068912)
const IN_PLACE_PTR = Ptr{Cvoid}(-1 % UInt)

# ---------------------------------------------------------------------------
# device buffer (north-star subsystem 1): HBM allocation owned by Julia
# ---------------------------------------------------------------------------
mutable struct ROCBuffer{T,N} <: AbstractArray{T,N}
    ptr::Ptr{T}
    dims::NTuple{N,Int}
    function ROCBuffer{T,N}(::UndefInitializer, dims::NTuple{N,Int}) where {T,N}
        p = Ref{Ptr{Cvoid}}(C_NULL)
        @mpichk ccall((:mpigx_malloc, libmpigx), Cint, (Ptr{Ptr{Cvoid}}, Csize_t), p, max(1, prod(dims)) * sizeof(T))
        b = new{T,N}(Ptr{T}(p[]), dims)
        finalizer(x -> ccall((:mpigx_free, libmpigx), Cint, (Ptr{Cvoid},), x.ptr), b)
        return b
    end
end
ROCBuffer{T}(::UndefInitializer, dims::Integer...) where {T} = ROCBuffer{T,length(dims)}(undef, Tuple(Int.(dims)))
function ROCBuffer(a::Array{T,N}) where {T,N}
    b = ROCBuffer{T,N}(undef, size(a))
    ccall((:mpigx_memcpy, libmpigx), Cint, (Ptr{Cvoid}, Ptr{Cvoid}, Csize_t), b.ptr, a, sizeof(a))
    return b
end
Base.size(b::ROCBuffer) = b.dims
Base.similar(b::ROCBuffer{T}, ::Type{S}, dims::Dims) where {T,S} = ROCBuffer{S,length(dims)}(undef, dims)
function Base.Array(b::ROCBuffer{T,N}) where {T,N}
    a = Array{T,N}(undef, b.dims)
    ccall((:mpigx_memcpy, libmpigx), Cint, (Ptr{Cvoid}, Ptr{Cvoid}, Csize_t), a, b.ptr, sizeof(a))
    return a
end
function Base.getindex(b::ROCBuffer{T}, i::Int) where T   # one element, host copy (tests)
    @boundscheck checkbounds(b, i)
    r = Ref{T}()
    ccall((:mpigx_memcpy, libmpigx), Cint, (Ptr{T}, Ptr{T}, Csize_t), r, b.ptr + (i - 1) * sizeof(T), sizeof(T))
    r[]
end
Base.:(==)(a::ROCBuffer, b::AbstractArray) = Array(a) == b
Base.cconvert(::Type{MPIPtr}, b::ROCBuffer) = b
Base.unsafe_convert(::Type{MPIPtr}, b::ROCBuffer) = reinterpret(MPIPtr, b.ptr)

const DeviceBuf = ROCBuffer
const DeviceOrSentinel = Union{ROCBuffer,SentinelPtr}

# ---------------------------------------------------------------------------
# engine communicators, created collectively on first device use of a Comm;
# the 128-byte unique id travels over host MPI (MPI.Bcast!)
# ---------------------------------------------------------------------------
# Keyed by the Comm OBJECT's identity (objectid), not by its handle value or
# by `==`: MPICH hands a freed communicator's handle value to the next new
# one, which must not inherit a stale engine communicator, and MPI.jl's Comm
# defines `==` by handle value (src/handle.jl:29-31) while keeping the
# identity hash, so a Dict/WeakKeyDict keyed by Comm mixes the two (after
# MPI.free every freed Comm `==` every other).  Each entry keeps a WeakRef to
# its Comm: an objectid reused by a later Comm (the old one collected) finds
# an entry whose ref is no longer that object, and drops it.
#
# Release (like comm.jl:85 `finalizer(free, newcomm)`): the Comm's GC
# finalizer releases its engine communicator locally (mpigx_comm_release: no
# barrier, safe once this rank's last collective on it returned).  A
# finalizer runs inside whatever task allocated, possibly one that holds
# ENGINE_LOCK, so it takes no lock and touches no Dict: it flips the entry's
# atomic `released` flag (whoever flips it first — the finalizer or
# __finalize at exit — does the release, exactly once) and engine() purges
# released or collected entries under the lock.  MPI.free(comm) sets comm.val
# to COMM_NULL, after which engine(comm) refuses the Comm.
mutable struct EngineEntry
    ref::WeakRef
    handle::Ptr{Cvoid}
    released::Threads.Atomic{Bool}
end
const ENGINE = Dict{UInt,EngineEntry}()
const ENGINE_LOCK = ReentrantLock()

function _engine_release(e::EngineEntry)
    if !Threads.atomic_cas!(e.released, false, true)
        ccall((:mpigx_comm_release, libmpigx), Cint, (Ptr{Cvoid},), e.handle)
        MPI.refcount_dec()
    end
    nothing
end

# engine(comm): the lock guards only the Dict (lookup, purge, insert).  The
# creation itself is collective — the unique id's MPI.Bcast!, the
# Comm_split_type, and mpigx_comm_init_rank's shm rendezvous with every rank —
# and runs WITHOUT the lock (VERDICT r05 item 5): held across it, two threads
# whose first device calls are on communicators X and Y could deadlock, rank 0
# taking the lock for X and waiting in X's Bcast! for rank 1, which holds it
# for Y and waits in Y's (legal under THREAD_MULTIPLE; the reference's
# Comm_dup / Comm_split, comm.jl:78-105, take no process-wide lock either).
# Two threads creating an engine for the SAME Comm at once would be two
# concurrent collectives on one communicator, which MPI forbids; should it
# happen, the second insert finds the first entry, keeps it and releases its
# own communicator.
function _engine_lookup(key, comm)
    e = get(ENGINE, key, nothing)
    if e !== nothing && (e.ref.value !== comm || e.released[])
        delete!(ENGINE, key)  # another (collected) Comm's entry at a reused objectid
        e = nothing
    end
    e
end

function engine(comm::Comm)
    comm.val == MPI.COMM_NULL.val && throw(MPI.MPIError(Cint(5)))  # MPI_ERR_COMM (MPICH mpi.h): a freed Comm
    key = objectid(comm)
    e = lock(ENGINE_LOCK) do
        _engine_lookup(key, comm)
    end
    e === nothing || return e.handle
    # collective creation, no lock held
    id = zeros(UInt8, 128)
    rank = MPI.Comm_rank(comm)
    if rank == 0
        @mpichk ccall((:mpigx_get_unique_id, libmpigx), Cint, (Ptr{UInt8},), id)
    end
    MPI.Bcast!(id, 0, comm)
    # rank -> GPU binding: node-local rank (comm.jl:107 Comm_split_type SHARED)
    local_comm = MPI.Comm_split_type(comm, MPI.MPI_COMM_TYPE_SHARED, rank)
    local_rank = MPI.Comm_rank(local_comm)
    MPI.free(local_comm)  # only its rank is needed (comm.jl:107)
    device = parse(Int, get(ENV, "MPIGX_DEVICE", string(local_rank)))
    h = Ref{Ptr{Cvoid}}(C_NULL)
    @mpichk ccall((:mpigx_comm_init_rank, libmpigx), Cint, (Ptr{Ptr{Cvoid}}, Cint, Ptr{UInt8}, Cint, Cint),
                  h, MPI.Comm_size(comm), id, rank, device)
    mine = EngineEntry(WeakRef(comm), h[], Threads.Atomic{Bool}(false))
    MPI.refcount_inc()  # released before MPI_Finalize (refcount_dec in _engine_release)
    # publish under the lock (purging released / collected entries on the way)
    winner = lock(ENGINE_LOCK) do
        filter!(kv -> kv.second.ref.value !== nothing && !kv.second.released[], ENGINE)
        other = _engine_lookup(key, comm)
        other === nothing || return other
        ENGINE[key] = mine
        mine
    end
    if winner !== mine
        _engine_release(mine)  # another thread's engine for this Comm came first (see above)
        return winner.handle
    end
    if !(comm === MPI.COMM_WORLD || comm === MPI.COMM_SELF)
        finalizer(_ -> _engine_release(mine), comm)  # lock-free (see above)
    end
    mine.handle
end

# ---------------------------------------------------------------------------
# datatype extension (datatypes.jl:281-284 would map BFloat16 to UINT16_T)
# ---------------------------------------------------------------------------
if isdefined(Main, :BFloat16s)
    Datatype(::Type{Main.BFloat16s.BFloat16}; commit=true) = MPI._Datatype(MPIGX_BFLOAT16)
end

# ---------------------------------------------------------------------------
# collectives: the reference signatures, ccall target swapped
# ---------------------------------------------------------------------------
# collective.jl:29-37
function Bcast!(buffer::ROCBuffer, count::Integer, root::Integer, comm::Comm)
    @mpichk ccall((:mpigx_bcast, libmpigx), Cint, (MPIPtr, Cint, MPI_Datatype, Cint, Ptr{Cvoid}),
                  buffer, count, Datatype(eltype(buffer)), root, engine(comm))
    buffer
end

# collective.jl:295-307
function Allgather!(sendbuf::DeviceOrSentinel, recvbuf::ROCBuffer, count::Integer, comm::Comm)
    MPI.@assert_minlength recvbuf count*MPI.Comm_size(comm)
    MPI.@assert_minlength sendbuf count
    T = eltype(recvbuf)
    @mpichk ccall((:mpigx_allgather, libmpigx), Cint,
                  (MPIPtr, Cint, MPI_Datatype, MPIPtr, Cint, MPI_Datatype, Ptr{Cvoid}),
                  sendbuf, count, Datatype(T), recvbuf, count, Datatype(T), engine(comm))
    recvbuf
end

# collective.jl:489-501
function Alltoall!(sendbuf::DeviceOrSentinel, recvbuf::ROCBuffer, count::Integer, comm::Comm)
    buflength = count * MPI.Comm_size(comm)
    MPI.@assert_minlength recvbuf buflength
    MPI.@assert_minlength sendbuf buflength
    sendbuf isa SentinelPtr || @assert eltype(sendbuf) == eltype(recvbuf)
    T = eltype(recvbuf)
    @mpichk ccall((:mpigx_alltoall, libmpigx), Cint,
                  (MPIPtr, Cint, MPI_Datatype, MPIPtr, Cint, MPI_Datatype, Ptr{Cvoid}),
                  sendbuf, count, Datatype(T), recvbuf, count, Datatype(T), engine(comm))
    recvbuf
end

# ---------------------------------------------------------------------------
# op handles on the engine (collective.jl:698-700 passes `op` straight to
# libmpi): built-in handles are the same MPICH values in both libraries; an
# `MPI.Op(f, T)` made by the REFERENCE (operators.jl:72-88) holds a libmpi
# handle from MPI_Op_create plus, in `fptr`, the @cfunction of its OpWrapper
# — an MPI_User_function, exactly what mpigx_op_create takes.  Such an op is
# re-registered with libmpigx once (commutativity from libmpi's
# MPI_Op_commutative) and the engine handle is cached for the Op's lifetime.
# libmpigx's own handles (DeviceOp below, csrc/handles.hpp space
# 0x3c000000) pass through; a foreign handle with no function (fptr ===
# nothing) is passed as is and libmpigx rejects it with MPI_ERR_OP.
# ---------------------------------------------------------------------------
const ENGINE_OPS = IdDict{Op,Cint}()
is_engine_handle(v) = (UInt32(reinterpret(UInt32, Cint(v))) & 0xfc000000) == 0x3c000000
function engine_op(op::Op)
    (op.fptr === nothing || is_engine_handle(op.val)) && return Cint(op.val)
    get!(ENGINE_OPS, op) do
        commute = Ref{Cint}(0)
        @mpichk ccall((:MPI_Op_commutative, MPI.libmpi), Cint, (MPI_Op, Ptr{Cint}), op.val, commute)
        h = Ref{Cint}(0)
        @mpichk ccall((:mpigx_op_create, libmpigx), Cint, (Ptr{Cvoid}, Cint, Ptr{Cint}),
                      Base.unsafe_convert(Ptr{Cvoid}, op.fptr), commute[], h)
        # the engine handle goes when the reference's Op is freed (operators.jl:47-53)
        finalizer(o -> (h2 = Ref(pop!(ENGINE_OPS, o, Cint(0))); h2[] != 0 &&
                        ccall((:mpigx_op_free, libmpigx), Cint, (Ptr{Cint},), h2)), op)
        h[]
    end
end
engine_op(op::MPI_Op) = Cint(op)

# collective.jl:605-618 (recvbuf may be `nothing` on non-roots)
function Reduce!(sendbuf::DeviceOrSentinel, recvbuf::Union{ROCBuffer,Nothing}, count::Integer,
                 op::Union{Op,MPI_Op}, root::Integer, comm::Comm)
    isroot = MPI.Comm_rank(comm) == root
    MPI.@assert_minlength sendbuf count
    if isroot
        @assert recvbuf !== nothing
        MPI.@assert_minlength recvbuf count
    end
    T = sendbuf isa SentinelPtr ? eltype(recvbuf) : eltype(sendbuf)
    @mpichk ccall((:mpigx_reduce, libmpigx), Cint,
                  (MPIPtr, MPIPtr, Cint, MPI_Datatype, MPI_Op, Cint, Ptr{Cvoid}),
                  sendbuf, recvbuf, count, Datatype(T), engine_op(op), root, engine(comm))
    recvbuf
end

# collective.jl:691-701
function Allreduce!(sendbuf::DeviceOrSentinel, recvbuf::ROCBuffer, count::Integer,
                    op::Union{Op,MPI_Op}, comm::Comm)
    MPI.@assert_minlength sendbuf count
    MPI.@assert_minlength recvbuf count
    sendbuf isa SentinelPtr || @assert eltype(sendbuf) == eltype(recvbuf)
    T = eltype(recvbuf)
    @mpichk ccall((:mpigx_allreduce, libmpigx), Cint,
                  (MPIPtr, MPIPtr, Cint, MPI_Datatype, MPI_Op, Ptr{Cvoid}),
                  sendbuf, recvbuf, count, Datatype(T), engine_op(op), engine(comm))
    recvbuf
end

# collective.jl:760-768 / :834-842
for (jl, c) in ((:Scan!, :mpigx_scan), (:Exscan!, :mpigx_exscan))
    @eval function $jl(sendbuf::DeviceOrSentinel, recvbuf::ROCBuffer, count::Integer,
                       op::Union{Op,MPI_Op}, comm::Comm)
        T = eltype(recvbuf)
        @mpichk ccall(($(QuoteNode(c)), libmpigx), Cint,
                      (MPIPtr, MPIPtr, Cint, MPI_Datatype, MPI_Op, Ptr{Cvoid}),
                      sendbuf, recvbuf, count, Datatype(T), engine_op(op), engine(comm))
        recvbuf
    end
end

# ---------------------------------------------------------------------------
# function-valued ops on device buffers: the reference's generic methods
# (collective.jl:703-705 Allreduce!, :622-625 Reduce!, :770-772 Scan!,
# :844-846 Exscan!) turn `opfunc` into MPI.Op(opfunc, T) — which for a
# non-builtin function calls MPI_Op_create in LIBMPI (operators.jl:72-88).  A
# libmpi op handle means nothing to libmpigx (its own handles live elsewhere,
# csrc/handles.hpp, and a foreign one is rejected with MPI_ERR_OP), so for
# ROCBuffers the function goes through device_op: the built-in mapping of
# operators.jl:39-45 (min/max/+/* on integer and float types, + and * on
# complex, &/|/⊻ on integers), anything else a libmpigx user op (DeviceOp).
# ---------------------------------------------------------------------------
const _MPIInteger = Union{Int8,UInt8,Int16,UInt16,Int32,UInt32,Int64,UInt64}
const _MPIFloat = Union{Float32,Float64}
const _MPIComplex = Union{ComplexF32,ComplexF64}
_is_bf16(::Type{T}) where T = isdefined(Main, :BFloat16s) && T === Main.BFloat16s.BFloat16

builtin_op(f, ::Type{T}) where T = nothing
for (fn, op, types) in ((min, :MIN, :(Union{_MPIInteger,_MPIFloat})),
                        (max, :MAX, :(Union{_MPIInteger,_MPIFloat})),
                        (+, :SUM, :(Union{_MPIInteger,_MPIFloat,_MPIComplex})),
                        (*, :PROD, :(Union{_MPIInteger,_MPIFloat,_MPIComplex})),
                        (&, :BAND, :_MPIInteger), (|, :BOR, :_MPIInteger), (⊻, :BXOR, :_MPIInteger))
    @eval builtin_op(::typeof($fn), ::Type{T}) where {T<:$types} = MPI.$op
end
function builtin_op(f, ::Type{T}) where T
    # bf16 (libmpigx extension): like the float types
    _is_bf16(T) || return nothing
    f === min ? MPI.MIN : f === max ? MPI.MAX : f === (+) ? MPI.SUM : f === (*) ? MPI.PROD : nothing
end

# (op, owned): owned user ops are freed after the call
function device_op(opfunc, ::Type{T}) where T
    opfunc isa Op && return (opfunc, false)
    b = builtin_op(opfunc, T)
    b !== nothing && return (b, false)
    (DeviceOp(opfunc, T), true)
end
function _with_device_op(f, opfunc, ::Type{T}) where T
    op, owned = device_op(opfunc, T)
    try
        return f(op)
    finally
        owned && ccall((:mpigx_op_free, libmpigx), Cint, (Ptr{Cint},), Ref(op.val))
    end
end

Allreduce!(sendbuf::DeviceOrSentinel, recvbuf::ROCBuffer, count::Integer, opfunc, comm::Comm) =
    _with_device_op(op -> Allreduce!(sendbuf, recvbuf, count, op, comm), opfunc, eltype(recvbuf))
function Reduce!(sendbuf::DeviceOrSentinel, recvbuf::Union{ROCBuffer,Nothing}, count::Integer, opfunc,
                 root::Integer, comm::Comm)
    T = sendbuf isa SentinelPtr ? eltype(recvbuf) : eltype(sendbuf)
    _with_device_op(op -> Reduce!(sendbuf, recvbuf, count, op, root, comm), opfunc, T)
end
Scan!(sendbuf::DeviceOrSentinel, recvbuf::ROCBuffer, count::Integer, opfunc, comm::Comm) =
    _with_device_op(op -> Scan!(sendbuf, recvbuf, count, op, comm), opfunc, eltype(recvbuf))
Exscan!(sendbuf::DeviceOrSentinel, recvbuf::ROCBuffer, count::Integer, opfunc, comm::Comm) =
    _with_device_op(op -> Exscan!(sendbuf, recvbuf, count, op, comm), opfunc, eltype(recvbuf))
# the reference's length-taking and in-place forms (collective.jl:707-714,
# :626-638, :773-783, :847-857) reach the methods above through dispatch on
# ROCBuffer; its in-place Scan!/Exscan! forms reference the undefined
# `sendbuf` (SURVEY §2 reference bugs) — here they work:
Scan!(buf::ROCBuffer, count::Integer, opfunc, comm::Comm) = Scan!(MPI.IN_PLACE, buf, count, opfunc, comm)
Scan!(buf::ROCBuffer, opfunc, comm::Comm) = Scan!(MPI.IN_PLACE, buf, length(buf), opfunc, comm)
Exscan!(buf::ROCBuffer, count::Integer, opfunc, comm::Comm) = Exscan!(MPI.IN_PLACE, buf, count, opfunc, comm)
Exscan!(buf::ROCBuffer, opfunc, comm::Comm) = Exscan!(MPI.IN_PLACE, buf, length(buf), opfunc, comm)

"""
    has_rocm()

The ROCm counterpart of `MPI.has_cuda()` (src/environment.jl:308-323), which
test/test_basic.jl gates the device test mode on: `JULIA_MPI_HAS_ROCM`
(true/false) overrides; otherwise true when libmpigx loads and a ROCm device
is visible to it.
"""
function has_rocm()
    flag = get(ENV, "JULIA_MPI_HAS_ROCM", nothing)
    flag === nothing || return parse(Bool, flag)
    try
        p = Ref{Ptr{Cvoid}}(C_NULL)
        ccall((:mpigx_malloc, libmpigx), Cint, (Ptr{Ptr{Cvoid}}, Csize_t), p, 16) == 0 || return false
        ccall((:mpigx_free, libmpigx), Cint, (Ptr{Cvoid},), p[])
        return true
    catch
        return false
    end
end

# ---------------------------------------------------------------------------
# point-to-point (src/pointtopoint.jl) on device buffers.  libmpigx requests
# are MPICH-style Cint handles; they live in their own type so Wait!/Test!
# dispatch to libmpigx without overwriting MPI.jl's Request methods.
# ---------------------------------------------------------------------------
import MPI: Send, Isend, Recv!, Irecv!, Sendrecv!, Wait!, Test!, Waitall!, Testall!, Waitany!,
            Cancel!, Buffer, Status, MPI_Request, STATUS_EMPTY

const DevBuffer = Buffer{<:ROCBuffer}
const MPIGX_REQUEST_NULL = Cint(0x2c000000)
const MPIGX_UNDEFINED = Cint(-32766)

mutable struct ROCRequest
    val::Cint
    buffer::Any
end
ROCRequest() = ROCRequest(MPIGX_REQUEST_NULL, nothing)
isnull(r::ROCRequest) = r.val == MPIGX_REQUEST_NULL
function free(r::ROCRequest)
    if !isnull(r)
        ccall((:mpigx_request_free, libmpigx), Cint, (Ptr{Cint},), Ref(r.val))
        r.val = MPIGX_REQUEST_NULL
        r.buffer = nothing
    end
end

# pointtopoint.jl:188-198
function Send(buf::DevBuffer, dest::Integer, tag::Integer, comm::Comm)
    @mpichk ccall((:mpigx_send, libmpigx), Cint,
                  (MPIPtr, Cint, MPI_Datatype, Cint, Cint, Ptr{Cvoid}),
                  buf.data, buf.count, buf.datatype, dest, tag, engine(comm))
    nothing
end
# pointtopoint.jl:221-236
function Isend(buf::DevBuffer, dest::Integer, tag::Integer, comm::Comm)
    h = Ref{Cint}(MPIGX_REQUEST_NULL)
    @mpichk ccall((:mpigx_isend, libmpigx), Cint,
                  (MPIPtr, Cint, MPI_Datatype, Cint, Cint, Ptr{Cvoid}, Ptr{Cint}),
                  buf.data, buf.count, buf.datatype, dest, tag, engine(comm), h)
    req = ROCRequest(h[], buf)
    finalizer(free, req)
    req
end
# pointtopoint.jl:266-276
function Recv!(buf::DevBuffer, src::Integer, tag::Integer, comm::Comm)
    stat_ref = Ref{Status}(STATUS_EMPTY)
    @mpichk ccall((:mpigx_recv, libmpigx), Cint,
                  (MPIPtr, Cint, MPI_Datatype, Cint, Cint, Ptr{Cvoid}, Ptr{Status}),
                  buf.data, buf.count, buf.datatype, src, tag, engine(comm), stat_ref)
    stat_ref[]
end
# pointtopoint.jl:325-339
function Irecv!(buf::DevBuffer, src::Integer, tag::Integer, comm::Comm)
    h = Ref{Cint}(MPIGX_REQUEST_NULL)
    @mpichk ccall((:mpigx_irecv, libmpigx), Cint,
                  (MPIPtr, Cint, MPI_Datatype, Cint, Cint, Ptr{Cvoid}, Ptr{Cint}),
                  buf.data, buf.count, buf.datatype, src, tag, engine(comm), h)
    req = ROCRequest(h[], buf)
    finalizer(free, req)
    req
end
# pointtopoint.jl:370-391
function Sendrecv!(sendbuf::DevBuffer, dest::Integer, sendtag::Integer,
                   recvbuf::DevBuffer, source::Integer, recvtag::Integer, comm::Comm)
    stat_ref = Ref{Status}(STATUS_EMPTY)
    @mpichk ccall((:mpigx_sendrecv, libmpigx), Cint,
                  (MPIPtr, Cint, MPI_Datatype, Cint, Cint, MPIPtr, Cint, MPI_Datatype, Cint, Cint,
                   Ptr{Cvoid}, Ptr{Status}),
                  sendbuf.data, sendbuf.count, sendbuf.datatype, dest, sendtag,
                  recvbuf.data, recvbuf.count, recvbuf.datatype, source, recvtag, engine(comm), stat_ref)
    stat_ref[]
end
# pointtopoint.jl:398-417 (returns the Status; the reference returns `stat`, a typo)
function Wait!(req::ROCRequest)
    stat_ref = Ref{Status}(STATUS_EMPTY)
    h = Ref(req.val)
    @mpichk ccall((:mpigx_wait, libmpigx), Cint, (Ptr{Cint}, Ptr{Status}), h, stat_ref)
    req.val = h[]; req.buffer = nothing
    stat_ref[]
end
# pointtopoint.jl:427-446
function Test!(req::ROCRequest)
    flag = Ref{Cint}(0); stat_ref = Ref{Status}(STATUS_EMPTY); h = Ref(req.val)
    @mpichk ccall((:mpigx_test, libmpigx), Cint, (Ptr{Cint}, Ptr{Cint}, Ptr{Status}), h, flag, stat_ref)
    flag[] == 0 && return (false, nothing)
    req.val = h[]; req.buffer = nothing
    (true, stat_ref[])
end
# pointtopoint.jl:457-477
function Waitall!(reqs::Vector{ROCRequest})
    vals = [r.val for r in reqs]; stats = fill(STATUS_EMPTY, length(reqs))
    @mpichk ccall((:mpigx_waitall, libmpigx), Cint, (Cint, Ptr{Cint}, Ptr{Status}), length(reqs), vals, stats)
    for (r, v) in zip(reqs, vals); r.val = v; r.buffer = nothing; end
    stats
end
# pointtopoint.jl:490-514
function Testall!(reqs::Vector{ROCRequest})
    vals = [r.val for r in reqs]; flag = Ref{Cint}(0); stats = fill(STATUS_EMPTY, length(reqs))
    @mpichk ccall((:mpigx_testall, libmpigx), Cint, (Cint, Ptr{Cint}, Ptr{Cint}, Ptr{Status}),
                  length(reqs), vals, flag, stats)
    flag[] == 0 && return (false, nothing)
    for (r, v) in zip(reqs, vals); r.val = v; r.buffer = nothing; end
    (true, stats)
end
# pointtopoint.jl:527-546
function Waitany!(reqs::Vector{ROCRequest})
    vals = [r.val for r in reqs]; ind = Ref{Cint}(); stat_ref = Ref{Status}(STATUS_EMPTY)
    @mpichk ccall((:mpigx_waitany, libmpigx), Cint, (Cint, Ptr{Cint}, Ptr{Cint}, Ptr{Status}),
                  length(reqs), vals, ind, stat_ref)
    ind[] == MPIGX_UNDEFINED && return (0, stat_ref[])
    i = Int(ind[]) + 1
    reqs[i].val = vals[i]; reqs[i].buffer = nothing
    (i, stat_ref[])
end
# pointtopoint.jl:671-681
function Cancel!(req::ROCRequest)
    @mpichk ccall((:mpigx_cancel, libmpigx), Cint, (Ptr{Cint},), Ref(req.val))
    nothing
end

# ---------------------------------------------------------------------------
# one-sided (src/onesided.jl) on device windows.  libmpigx windows are
# opaque pointers; ROCWin keeps them apart from MPI.Win so the reference's
# host methods stay untouched.
# ---------------------------------------------------------------------------
import MPI: Win_create, Win_create_dynamic, Win_fence, Win_flush, Win_sync, Win_lock, Win_unlock,
            Win_attach, Win_detach, Get, Put, Fetch_and_op, Accumulate, Get_accumulate, LockType

mutable struct ROCWin
    ptr::Ptr{Cvoid}
    comm::Comm
end
function wfree(w::ROCWin)
    if w.ptr != C_NULL
        h = Ref(w.ptr)
        @mpichk ccall((:mpigx_win_free, libmpigx), Cint, (Ptr{Ptr{Cvoid}},), h)
        w.ptr = C_NULL
    end
end
MPI.free(w::ROCWin) = wfree(w)

# onesided.jl:24-34
function Win_create(base::ROCBuffer{T}, comm::Comm; infokws...) where T
    h = Ref{Ptr{Cvoid}}(C_NULL)
    @mpichk ccall((:mpigx_win_create, libmpigx), Cint, (Ptr{Cvoid}, Clonglong, Cint, Ptr{Cvoid}, Ptr{Ptr{Cvoid}}),
                  base.ptr, length(base) * sizeof(T), sizeof(T), engine(comm), h)
    w = ROCWin(h[], comm); finalizer(wfree, w); w
end
# onesided.jl:47-56 (device flavour: `Win_create_dynamic(ROCBuffer, comm)`)
function Win_create_dynamic(::Type{ROCBuffer}, comm::Comm; kwargs...)
    h = Ref{Ptr{Cvoid}}(C_NULL)
    @mpichk ccall((:mpigx_win_create_dynamic, libmpigx), Cint, (Ptr{Cvoid}, Ptr{Ptr{Cvoid}}), engine(comm), h)
    w = ROCWin(h[], comm); finalizer(wfree, w); w
end
# onesided.jl:72-83 (device flavour): returns (win, device pointer)
function Win_allocate_shared(::Type{ROCBuffer}, ::Type{T}, len::Int, comm::Comm; kwargs...) where T
    h = Ref{Ptr{Cvoid}}(C_NULL); p = Ref{Ptr{T}}(C_NULL)
    @mpichk ccall((:mpigx_win_allocate_shared, libmpigx), Cint,
                  (Clonglong, Cint, Ptr{Cvoid}, Ptr{Ptr{T}}, Ptr{Ptr{Cvoid}}), len * sizeof(T), sizeof(T), engine(comm), p, h)
    w = ROCWin(h[], comm); finalizer(wfree, w); (w, p[])
end
function Win_shared_query(w::ROCWin, owner_rank::Int)
    len = Ref{Clonglong}(); du = Ref{Cint}(); p = Ref{Ptr{Cvoid}}()
    @mpichk ccall((:mpigx_win_shared_query, libmpigx), Cint, (Ptr{Cvoid}, Cint, Ptr{Clonglong}, Ptr{Cint}, Ptr{Ptr{Cvoid}}),
                  w.ptr, owner_rank, len, du, p)
    len[], du[], p[]
end
Win_attach(w::ROCWin, base::ROCBuffer{T}) where T =
    @mpichk ccall((:mpigx_win_attach, libmpigx), Cint, (Ptr{Cvoid}, Ptr{Cvoid}, Clonglong), w.ptr, base.ptr, sizeof(T) * length(base))
Win_detach(w::ROCWin, base::ROCBuffer) =
    @mpichk ccall((:mpigx_win_detach, libmpigx), Cint, (Ptr{Cvoid}, Ptr{Cvoid}), w.ptr, base.ptr)
# onesided.jl:124-148
Win_fence(assert::Integer, w::ROCWin) = @mpichk ccall((:mpigx_win_fence, libmpigx), Cint, (Cint, Ptr{Cvoid}), assert, w.ptr)
Win_flush(rank::Integer, w::ROCWin) = @mpichk ccall((:mpigx_win_flush, libmpigx), Cint, (Cint, Ptr{Cvoid}), rank, w.ptr)
Win_sync(w::ROCWin) = @mpichk ccall((:mpigx_win_sync, libmpigx), Cint, (Ptr{Cvoid},), w.ptr)
Win_lock(lt::LockType, rank::Integer, assert::Integer, w::ROCWin) =
    @mpichk ccall((:mpigx_win_lock, libmpigx), Cint, (Cint, Cint, Cint, Ptr{Cvoid}), lt.val, rank, assert, w.ptr)
Win_unlock(rank::Integer, w::ROCWin) = @mpichk ccall((:mpigx_win_unlock, libmpigx), Cint, (Cint, Ptr{Cvoid}), rank, w.ptr)
# onesided.jl:150-184 (device origin buffers)
for (jl, c) in ((:Get, :mpigx_get), (:Put, :mpigx_put))
    @eval function $jl(origin::ROCBuffer{T}, count::Integer, target_rank::Integer, target_disp::Integer, w::ROCWin) where T
        @mpichk ccall(($(QuoteNode(c)), libmpigx), Cint,
                      (MPIPtr, Cint, MPI_Datatype, Cint, Clonglong, Cint, MPI_Datatype, Ptr{Cvoid}),
                      origin, count, Datatype(T), target_rank, target_disp, count, Datatype(T), w.ptr)
    end
    @eval $jl(origin::ROCBuffer, target_rank::Integer, w::ROCWin) = $jl(origin, length(origin), target_rank, 0, w)
end
# onesided.jl:186-195
function Fetch_and_op(sourceval::ROCBuffer{T}, returnval::ROCBuffer{T}, target_rank::Integer,
                      target_disp::Integer, op::Op, w::ROCWin) where T
    @mpichk ccall((:mpigx_fetch_and_op, libmpigx), Cint,
                  (MPIPtr, MPIPtr, MPI_Datatype, Cint, Clonglong, MPI_Op, Ptr{Cvoid}),
                  sourceval, returnval, Datatype(T), target_rank, target_disp, op, w.ptr)
end
# onesided.jl:197-206
function Accumulate(origin::ROCBuffer{T}, count::Integer, target_rank::Integer, target_disp::Integer,
                    op::Op, w::ROCWin) where T
    @mpichk ccall((:mpigx_accumulate, libmpigx), Cint,
                  (MPIPtr, Cint, MPI_Datatype, Cint, Clonglong, Cint, MPI_Datatype, MPI_Op, Ptr{Cvoid}),
                  origin, count, Datatype(T), target_rank, target_disp, count, Datatype(T), op, w.ptr)
end
# onesided.jl:208-219
function Get_accumulate(origin::ROCBuffer{T}, result::ROCBuffer{T}, count::Integer, target_rank::Integer,
                        target_disp::Integer, op::Op, w::ROCWin) where T
    @mpichk ccall((:mpigx_get_accumulate, libmpigx), Cint,
                  (MPIPtr, Cint, MPI_Datatype, MPIPtr, Cint, MPI_Datatype, Cint, Clonglong, Cint, MPI_Datatype,
                   MPI_Op, Ptr{Cvoid}),
                  origin, count, Datatype(T), result, count, Datatype(T), target_rank, target_disp, count,
                  Datatype(T), op, w.ptr)
end

# ---------------------------------------------------------------------------
# derived datatypes for device buffers (datatypes.jl:62-318, buffers.jl:104-117):
# libmpigx keeps its own type table (handles in its own space, csrc/handles.hpp),
# so SubArrays of a ROCBuffer get libmpigx vector / subarray types.
# ---------------------------------------------------------------------------
module DevTypes
    import ..MPIGX: libmpigx
    import MPI: Datatype, MPI_Datatype, @mpichk
    dt(v::Cint) = MPI._Datatype(v)
    function create_vector(count, bl, stride, old::Datatype)
        r = Ref{Cint}()
        @mpichk ccall((:mpigx_type_vector, libmpigx), Cint, (Cint, Cint, Cint, Cint, Ptr{Cint}), count, bl, stride, old.val, r)
        dt(r[])
    end
    function create_subarray(sizes, subsizes, offset, old::Datatype; rowmajor=false)
        r = Ref{Cint}()
        @mpichk ccall((:mpigx_type_create_subarray, libmpigx), Cint,
                      (Cint, Ptr{Cint}, Ptr{Cint}, Ptr{Cint}, Cint, Cint, Ptr{Cint}),
                      length(sizes), Cint[sizes...], Cint[subsizes...], Cint[offset...], rowmajor ? 56 : 57, old.val, r)
        dt(r[])
    end
    function create_struct(bl, disp, types)
        r = Ref{Cint}()
        @mpichk ccall((:mpigx_type_create_struct, libmpigx), Cint, (Cint, Ptr{Cint}, Ptr{Clonglong}, Ptr{Cint}, Ptr{Cint}),
                      length(bl), Cint[bl...], Clonglong[disp...], Cint[t.val for t in types], r)
        dt(r[])
    end
    function commit!(d::Datatype)
        r = Ref(d.val)
        @mpichk ccall((:mpigx_type_commit, libmpigx), Cint, (Ptr{Cint},), r)
        d
    end
end
# buffers.jl:104-117 for views of device buffers
function Buffer(sub::SubArray{T,1,<:ROCBuffer}) where T
    stride1 = strides(sub)[1]
    d = DevTypes.commit!(DevTypes.create_vector(length(sub), 1, stride1, Datatype(T)))
    Buffer(sub, Cint(1), d)
end
function Buffer(sub::SubArray{T,N,<:ROCBuffer}) where {T,N}
    d = DevTypes.commit!(DevTypes.create_subarray(size(parent(sub)), map(length, sub.indices),
                                                  map(i -> first(i) - 1, sub.indices), Datatype(T)))
    Buffer(parent(sub), Cint(1), d)
end

# ---------------------------------------------------------------------------
# user-defined ops on device buffers (operators.jl:56-88): the reference's
# OpWrapper becomes an MPI_User_function that libmpigx calls on host-staged
# copies of the operands (mpigx_op_create).
# ---------------------------------------------------------------------------
function DeviceOp(f, ::Type{T}; iscommutative=false) where T
    w = MPI.OpWrapper{typeof(f),T}(f)
    fptr = @cfunction($w, Cvoid, (Ptr{Cvoid}, Ptr{Cvoid}, Ptr{Cint}, Ptr{MPI_Datatype}))
    r = Ref{Cint}()
    @mpichk ccall((:mpigx_op_create, libmpigx), Cint, (Ptr{Cvoid}, Cint, Ptr{Cint}), fptr, iscommutative, r)
    op = MPI.Op(r[], fptr)  # keeps the closure alive like operators.jl:85
    op
end

function __finalize()
    lock(ENGINE_LOCK) do
        for e in collect(values(ENGINE))
            _engine_release(e)  # skipped for entries a finalizer already released
        end
        empty!(ENGINE)
    end
end
# MPI.jl 0.14 has init hooks but no finalize hooks (environment.jl:26-62):
# engine communicators hold a refcount like any MPI object, so the libmpi
# finalizer runs after them (environment.jl:37-62, refcount_inc/_dec).
atexit(__finalize)

export ROCBuffer, ROCRequest, ROCWin, DeviceOp, has_rocm

end # module
