/*
 * Large-count golden vectors for the mpigx oracle (the
 * small-case fixtures stop at 1,100 elements, the headline runs 64 Mi).
 *
 * NOT product code and NOT part of the reference: it calls MPICH 3.3.2
 * (/opt/conda, the libmpi MPI.jl v0.14.2 ccalls) with the argument shapes of
 * src/collective.jl:615-617 (MPI_Reduce), :698-700 (MPI_Allreduce), :765-767
 * (MPI_Scan) and :839-841 (MPI_Exscan) at counts where MPICH runs its
 * large-message algorithms, and records SAMPLED SPANS of the outputs only
 * (the inputs are regenerated from the seeds by tests/gen_inputs.py
 * splitmix_input, so the fixture stays small):
 *   prefix, tail, and +-64 elements around every Rabenseifner block boundary
 *   k * (count / pof2) (where the owner of an element changes).
 *
 * Inputs: splitmix64 keyed by (case seed, rank, element index), the same
 * keying as gen_mpich_golden.c:
 *   f32 = ((r >> 40) - 2^23) / 2^23,  f64 = ((r >> 11) - 2^52) / 2^52,
 *   i64 = (int64) r;  "edge" cases replace the element with
 *   {+0, -0, +inf, -inf, NaN, 2^-149 (f32) / 2^-1074 (f64), 1, -1}[(r >> 4) & 7]
 *   when (r & 15) == 0.
 *
 * Run (tests/golden/make_large_golden.sh):  mpiexec -n {5,8} ./gen <outdir>
 * Each rank writes <outdir>/<case>.r<rank>.bin (its sampled output bytes,
 * spans concatenated); rank 0 writes <outdir>/manifest_large_<n>.jsonl.
 */
#include <math.h>
#include <mpi.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static uint64_t splitmix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}
static uint64_t key(uint64_t seed, int rank, uint64_t i) {
    return splitmix64(seed * 0x100000001B3ull ^ ((uint64_t)rank << 40) ^ i);
}

enum { K_F32 = 0, K_F64 = 1, K_I64 = 2 };

static void gen(int kind, int edge, uint64_t seed, int rank, long count, void *out) {
    static const double E[8] = {0.0, -0.0, INFINITY, -INFINITY, NAN, 0.0 /* denormal below */, 1.0, -1.0};
    for (long i = 0; i < count; ++i) {
        const uint64_t r = key(seed, rank, (uint64_t)i);
        if (kind == K_I64) {
            ((int64_t *)out)[i] = (int64_t)r;
        } else if (kind == K_F32) {
            float v = (float)((int64_t)(r >> 40) - (1ll << 23)) / (float)(1 << 23);
            if (edge && (r & 15) == 0) {
                const int e = (int)((r >> 4) & 7);
                v = e == 5 ? ldexpf(1.0f, -149) : (float)E[e];
            }
            ((float *)out)[i] = v;
        } else {
            double v = (double)((int64_t)(r >> 11) - (1ll << 52)) / 4503599627370496.0;
            if (edge && (r & 15) == 0) {
                const int e = (int)((r >> 4) & 7);
                v = e == 5 ? ldexp(1.0, -1074) : E[e];
            }
            ((double *)out)[i] = v;
        }
    }
}

static int pof2_of(int n) {
    int p = 1;
    while (p * 2 <= n) p *= 2;
    return p;
}

/* sampled spans [lo, hi): prefix, tail, around every block boundary */
static int spans(long count, int n, long *lo, long *hi) {
    const int pof2 = pof2_of(n);
    const long blk = count / pof2;
    int m = 0;
    lo[m] = 0, hi[m++] = 256;
    for (int k = 1; k < pof2; ++k) lo[m] = k * blk - 64, hi[m++] = k * blk + 64;
    lo[m] = count - 256, hi[m++] = count;
    return m;
}

typedef struct {
    const char *coll; /* allreduce | reduce | scan | exscan */
    int kind, edge;
    const char *dt;
    MPI_Datatype mdt;
    const char *opname;
    MPI_Op op;
    long count;
    uint64_t seed;
} Case;

int main(int argc, char **argv) {
    MPI_Init(&argc, &argv);
    int rank, n;
    MPI_Comm_rank(MPI_COMM_WORLD, &rank);
    MPI_Comm_size(MPI_COMM_WORLD, &n);
    const char *dir = argc > 1 ? argv[1] : ".";
    const long big = 4194307, mid = 1048579;
    const Case cases[] = {
        {"allreduce", K_F32, 0, "FLOAT", MPI_FLOAT, "SUM", MPI_SUM, big, 101},
        {"allreduce", K_F64, 0, "DOUBLE", MPI_DOUBLE, "SUM", MPI_SUM, big, 102},
        {"allreduce", K_F32, 1, "FLOAT", MPI_FLOAT, "MAX", MPI_MAX, big, 103},
        {"reduce", K_F32, 0, "FLOAT", MPI_FLOAT, "SUM", MPI_SUM, big, 104},
        {"reduce", K_F64, 0, "DOUBLE", MPI_DOUBLE, "SUM", MPI_SUM, big, 105},
        {"reduce", K_F32, 1, "FLOAT", MPI_FLOAT, "MAX", MPI_MAX, big, 106},
        {"scan", K_I64, 0, "INT64_T", MPI_INT64_T, "BOR", MPI_BOR, mid, 107},
        {"exscan", K_I64, 0, "INT64_T", MPI_INT64_T, "BOR", MPI_BOR, mid, 108},
        {"scan", K_F64, 0, "DOUBLE", MPI_DOUBLE, "SUM", MPI_SUM, mid, 109},
    };
    const int ncases = (int)(sizeof cases / sizeof cases[0]);
    FILE *man = NULL;
    if (rank == 0) {
        char p[1024];
        snprintf(p, sizeof p, "%s/manifest_large_%d.jsonl", dir, n);
        man = fopen(p, "w");
    }
    for (int c = 0; c < ncases; ++c) {
        const Case *C = &cases[c];
        const int es = C->kind == K_F32 ? 4 : 8;
        char *in = malloc((size_t)C->count * es), *out = malloc((size_t)C->count * es);
        gen(C->kind, C->edge, C->seed, rank, C->count, in);
        memset(out, 0xCD, (size_t)C->count * es);
        const int root = n - 1; /* reduce: the last rank (a non-zero root) */
        if (!strcmp(C->coll, "allreduce")) MPI_Allreduce(in, out, (int)C->count, C->mdt, C->op, MPI_COMM_WORLD);
        else if (!strcmp(C->coll, "reduce")) MPI_Reduce(in, out, (int)C->count, C->mdt, C->op, root, MPI_COMM_WORLD);
        else if (!strcmp(C->coll, "scan")) MPI_Scan(in, out, (int)C->count, C->mdt, C->op, MPI_COMM_WORLD);
        else MPI_Exscan(in, out, (int)C->count, C->mdt, C->op, MPI_COMM_WORLD);
        long lo[32], hi[32];
        const int m = spans(C->count, n, lo, hi);
        char id[256];
        snprintf(id, sizeof id, "large_n%d_%s_%s_%s%s", n, C->coll, C->dt, C->opname, C->edge ? "_edge" : "");
        const int writes = !strcmp(C->coll, "reduce") ? rank == root : !strcmp(C->coll, "allreduce") ? rank == 0 : 1;
        if (writes) {
            char p[1024];
            snprintf(p, sizeof p, "%s/%s.r%d.bin", dir, id, rank);
            FILE *f = fopen(p, "wb");
            for (int s = 0; s < m; ++s) fwrite(out + (size_t)lo[s] * es, es, (size_t)(hi[s] - lo[s]), f);
            fclose(f);
        }
        if (man) {
            fprintf(man, "{\"id\": \"%s\", \"coll\": \"%s\", \"n\": %d, \"dtype\": \"%s\", \"op\": \"%s\", "
                         "\"count\": %ld, \"seed\": %llu, \"edge\": %d, \"root\": %d, \"kind\": \"%s\", \"spans\": [",
                    id, C->coll, n, C->dt, C->opname, C->count, (unsigned long long)C->seed, C->edge,
                    !strcmp(C->coll, "reduce") ? root : 0, C->kind == K_F32 ? "f32" : C->kind == K_F64 ? "f64" : "i64");
            for (int s = 0; s < m; ++s) fprintf(man, "%s[%ld, %ld]", s ? ", " : "", lo[s], hi[s]);
            fprintf(man, "]}\n");
        }
        free(in);
        free(out);
    }
    if (man) fclose(man);
    MPI_Finalize();
    return 0;
}
