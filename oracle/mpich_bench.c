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
 *   sweep MAXMIB            BASELINE.md's CPU plan in one run (mpiexec -n N):
 *                           Allreduce f32 SUM 8 KiB..MAXMIB (collective.jl:
 *                           698-700), Bcast! / Allgather! / Alltoall! f32
 *                           64 KiB..2*MAXMIB (:34, :304, :498; S = the
 *                           Bcast buffer / the Allgather receive total / the
 *                           Alltoall send total), Scan! / Exscan! / Reduce!
 *                           Int32 / Int64 BAND / BOR / MAX at 1 Ki, 1 Mi and
 *                           16 Mi elements (:765, :839, :615); the max time
 *                           over ranks, nccl-tests busbw factors; messages
 *                           >= 16 MiB: 1-2 timed calls, no warm-up
 *
 * Prints one JSON line (rank 0): seconds per call, algorithmic GB/s, busbw.
 * Built by oracle/Makefile into oracle/_ref/mpich_bench.
 */
#include <mpi.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

/* one collective timed: warm-up, barrier, iters calls, max over ranks */
typedef void (*coll_fn)(void *s, void *r, int count, MPI_Datatype dt, MPI_Op op, int size);
static void c_allreduce(void *s, void *r, int n, MPI_Datatype dt, MPI_Op op, int size) {
    (void)size;
    MPI_Allreduce(s, r, n, dt, op, MPI_COMM_WORLD);
}
static void c_bcast(void *s, void *r, int n, MPI_Datatype dt, MPI_Op op, int size) {
    (void)r; (void)op; (void)size;
    MPI_Bcast(s, n, dt, 0, MPI_COMM_WORLD);
}
static void c_allgather(void *s, void *r, int n, MPI_Datatype dt, MPI_Op op, int size) {
    (void)op;
    MPI_Allgather(s, n / size, dt, r, n / size, dt, MPI_COMM_WORLD);
}
static void c_alltoall(void *s, void *r, int n, MPI_Datatype dt, MPI_Op op, int size) {
    (void)op;
    MPI_Alltoall(s, n / size, dt, r, n / size, dt, MPI_COMM_WORLD);
}
static void c_scan(void *s, void *r, int n, MPI_Datatype dt, MPI_Op op, int size) {
    (void)size;
    MPI_Scan(s, r, n, dt, op, MPI_COMM_WORLD);
}
static void c_exscan(void *s, void *r, int n, MPI_Datatype dt, MPI_Op op, int size) {
    (void)size;
    MPI_Exscan(s, r, n, dt, op, MPI_COMM_WORLD);
}
static void c_reduce(void *s, void *r, int n, MPI_Datatype dt, MPI_Op op, int size) {
    MPI_Reduce(s, r, n, dt, op, size - 1, MPI_COMM_WORLD);
}
static double time_coll(coll_fn f, void *s, void *r, int n, MPI_Datatype dt, MPI_Op op, int size, int iters,
                        int warm) {
    if (warm) f(s, r, n, dt, op, size); /* warm-up (small messages) */
    MPI_Barrier(MPI_COMM_WORLD);
    double t0 = MPI_Wtime();
    for (int it = 0; it < iters; it++) f(s, r, n, dt, op, size);
    double t = (MPI_Wtime() - t0) / iters, tmax;
    MPI_Allreduce(&t, &tmax, 1, MPI_DOUBLE, MPI_MAX, MPI_COMM_WORLD);
    return tmax;
}

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
    } else if (!strcmp(argv[1], "sweep")) {
        size_t maxmib = (size_t)atol(argv[2]);
        size_t maxb = (maxmib << 21); /* byte movers: up to 2 x MAXMIB */
        char *s = malloc(maxb), *r = malloc(maxb);
        for (size_t i = 0; i < maxb; i++) s[i] = (char)((i * 131 + rank) & 0x7f);
        memset(r, 0, maxb);
        const double f = (double)(size - 1) / size;
        if (!rank) printf("{\"mode\":\"sweep\",\"ranks\":%d", size);
        /* Allreduce f32 SUM: the GPU line's sweep sizes (bench.py) */
        const size_t ar_sizes[5] = {8 << 10, 1 << 20, 16 << 20, 64 << 20, 256 << 20};
        for (int k = 0; k < 5; k++) {
            const size_t b = ar_sizes[k];
            if (b > (maxmib << 20)) break;
            int big = b >= (16u << 20), it = big ? 2 : 20;
            double t = time_coll(c_allreduce, s, r, (int)(b / 4), MPI_FLOAT, MPI_SUM, size, it, !big);
            if (!rank) printf(",\"allreduce_%zuKiB\":{\"sec\":%.6g,\"algbw_GBps\":%.4f,\"busbw_GBps\":%.4f}", b >> 10, t,
                              b / t / 1e9, b / t / 1e9 * 2 * f);
        }
        /* Bcast / Allgather / Alltoall f32: config 4's sizes (bench.py) */
        const size_t mv_sizes[5] = {64 << 10, 1 << 20, 16 << 20, 128 << 20, 512 << 20};
        for (int k = 0; k < 5; k++) {
            const size_t b = mv_sizes[k];
            if (b > maxb) break;
            int big = b >= (16u << 20), it = big ? 1 : 10;
            int cnt = (int)(b / 4 / size * size);
            double tb = time_coll(c_bcast, s, r, (int)(b / 4), MPI_FLOAT, MPI_SUM, size, it, !big);
            double tg = time_coll(c_allgather, s, r, cnt, MPI_FLOAT, MPI_SUM, size, it, !big);
            double ta = time_coll(c_alltoall, s, r, cnt, MPI_FLOAT, MPI_SUM, size, it, !big);
            if (!rank)
                printf(",\"movers_%zuKiB\":{\"bcast_busbw_GBps\":%.4f,\"allgather_busbw_GBps\":%.4f,"
                       "\"alltoall_busbw_GBps\":%.4f}", b >> 10, b / tb / 1e9, b / tg / 1e9 * f, b / ta / 1e9 * f);
        }
        /* Scan / Exscan / Reduce, Int32 / Int64, BAND / BOR / MAX */
        MPI_Datatype dts[2] = {MPI_INT32_T, MPI_INT64_T};
        const char *dtn[2] = {"int32", "int64"};
        int es[2] = {4, 8};
        MPI_Op ops[3] = {MPI_BAND, MPI_BOR, MPI_MAX};
        const char *opn[3] = {"BAND", "BOR", "MAX"};
        /* config 5's counts, the largest bounded to 16 Mi elements (MPICH's
           Scan moves ~0.1 GB/s per rank on the host: 64 Mi Int64 would take
           minutes; the GPU line runs 64 Mi) */
        size_t counts[3] = {1 << 10, 1 << 20, 16 << 20};
        for (int d = 0; d < 2; d++)
            for (int c = 0; c < 3; c++) {
                size_t cnt = counts[c];
                if (cnt * es[d] > maxb) cnt = maxb / es[d];
                int big = cnt * es[d] >= (16u << 20), it = big ? 1 : 10;
                for (int o = 0; o < 3; o++) {
                    double ts = time_coll(c_scan, s, r, (int)cnt, dts[d], ops[o], size, it, !big);
                    double te = time_coll(c_exscan, s, r, (int)cnt, dts[d], ops[o], size, it, !big);
                    double tr = time_coll(c_reduce, s, r, (int)cnt, dts[d], ops[o], size, it, !big);
                    double B = (double)cnt * es[d];
                    if (!rank)
                        printf(",\"%s_%s_%zu\":{\"scan_algbw_GBps\":%.4f,\"exscan_algbw_GBps\":%.4f,"
                               "\"reduce_algbw_GBps\":%.4f}", dtn[d], opn[o], cnt, B / ts / 1e9, B / te / 1e9,
                               B / tr / 1e9);
                }
            }
        if (!rank) printf("}\n");
        free(s);
        free(r);
    }
    MPI_Finalize();
    return 0;
}
