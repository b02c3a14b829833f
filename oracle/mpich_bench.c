/*
 * CPU baseline harness (TEST/BENCH INFRASTRUCTURE ONLY — bench.py's
 * cpu_baseline leg).  Times the reference's own arithmetic: MPICH 3.3.2, the
 * libmpi MPI.jl v0.14.2 ccalls by default (Project.toml:10), called exactly
 * like MPI.jl's ccall sites do:
 *
 *   local  NBUF MIB ITERS   MPI_Reduce_local folding NBUF host buffers of
 *                           MIB MiB f32 SUM (the host counterpart of the
 *                           config-2 device kernel; BASELINE.md plan)
 *   allreduce MIB ITERS     MPI_Allreduce(send, recv, count, MPI_FLOAT,
 *                           MPI_SUM, MPI_COMM_WORLD) — collective.jl:698-700;
 *                           run under `mpiexec -n N`
 *
 * Prints one JSON line (rank 0): seconds per call, algorithmic GB/s, busbw.
 * Built by oracle/Makefile into oracle/_ref/mpich_bench.
 */
#include <mpi.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

int main(int argc, char **argv) {
    MPI_Init(&argc, &argv);
    int rank, size;
    MPI_Comm_rank(MPI_COMM_WORLD, &rank);
    MPI_Comm_size(MPI_COMM_WORLD, &size);
    if (argc < 2) {
        if (!rank) fprintf(stderr, "usage: mpich_bench local NBUF MIB ITERS | allreduce MIB ITERS\n");
        MPI_Abort(MPI_COMM_WORLD, 2);
    }
    if (!strcmp(argv[1], "local")) {
        int nbuf = atoi(argv[2]);
        size_t mib = (size_t)atol(argv[3]);
        int iters = atoi(argv[4]);
        size_t count = mib << 18; /* f32 elements */
        float **in = malloc(sizeof(float *) * nbuf);
        for (int k = 0; k < nbuf; k++) {
            in[k] = malloc(count * sizeof(float));
            for (size_t i = 0; i < count; i++) in[k][i] = (float)((i * 2654435761u + k) % 1000) * 1e-3f;
        }
        float *out = malloc(count * sizeof(float));
        double best = 1e30, tot = 0;
        for (int it = 0; it <= iters; it++) {
            double t0 = MPI_Wtime();
            memcpy(out, in[0], count * sizeof(float));
            for (int k = 1; k < nbuf; k++) {
                /* chunked so the int count argument stays in range */
                for (size_t off = 0; off < count; off += (size_t)1 << 30) {
                    size_t c = count - off < ((size_t)1 << 30) ? count - off : ((size_t)1 << 30);
                    MPI_Reduce_local(in[k] + off, out + off, (int)c, MPI_FLOAT, MPI_SUM);
                }
            }
            double t = MPI_Wtime() - t0;
            if (it > 0) { tot += t; if (t < best) best = t; } /* it 0 = warm-up */
        }
        double per = tot / iters;
        double algo = (double)(nbuf + 1) * count * sizeof(float);
        printf("{\"mode\":\"local\",\"nbuf\":%d,\"mib\":%zu,\"iters\":%d,\"sec_per_call\":%.6f,\"best\":%.6f,"
               "\"algo_GBps\":%.3f,\"checksum\":%.6e}\n",
               nbuf, mib, iters, per, best, algo / per / 1e9, (double)out[count / 3]);
    } else if (!strcmp(argv[1], "allreduce")) {
        size_t mib = (size_t)atol(argv[2]);
        int iters = atoi(argv[3]);
        size_t count = mib << 18;
        float *s = malloc(count * sizeof(float)), *r = malloc(count * sizeof(float));
        for (size_t i = 0; i < count; i++) s[i] = (float)((i + rank) % 97) * 0.01f;
        MPI_Allreduce(s, r, (int)count, MPI_FLOAT, MPI_SUM, MPI_COMM_WORLD); /* warm-up */
        MPI_Barrier(MPI_COMM_WORLD);
        double t0 = MPI_Wtime();
        for (int it = 0; it < iters; it++) MPI_Allreduce(s, r, (int)count, MPI_FLOAT, MPI_SUM, MPI_COMM_WORLD);
        double t = (MPI_Wtime() - t0) / iters, tmax;
        MPI_Reduce(&t, &tmax, 1, MPI_DOUBLE, MPI_MAX, 0, MPI_COMM_WORLD);
        if (!rank) {
            double S = (double)count * 4;
            printf("{\"mode\":\"allreduce\",\"ranks\":%d,\"mib\":%zu,\"iters\":%d,\"sec_per_call\":%.6f,"
                   "\"algbw_GBps\":%.4f,\"busbw_GBps\":%.4f}\n",
                   size, mib, iters, tmax, S / tmax / 1e9, S / tmax / 1e9 * 2.0 * (size - 1) / size);
        }
    }
    MPI_Finalize();
    return 0;
}
