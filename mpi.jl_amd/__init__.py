"""mpi.jl_amd — MI355X-native collective engine for MPI.jl.

Layout: csrc/ (HIP kernels + C-ABI runtime -> lib/libmpigx.so),
mpigx/ (Python mirror of MPI.jl's collective API over the C ABI),
julia/ (the ccall glue MPI.jl would load).  The directory name is not a
Python identifier; put `mpi.jl_amd/` on sys.path and `import mpigx`.
"""
