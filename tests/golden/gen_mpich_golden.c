/*
 * Golden-vector generator for the mpigx parity tests.
 *
 * This program is NOT part of the product and is NOT part of the reference.
 * It calls MPICH 3.3.2 (/opt/conda/lib/libmpi.so.12 — the libmpi that
 * MPI.jl v0.14.2 ccalls by default, Project.toml:10, deps/build.jl:139-152)
 * with exactly the argument shapes of the reference's ccall sites
 * (src/collective.jl:34, :304, :498, :615, :698, :765, :839) and records
 * inputs + outputs of every rank, so the CPU oracle (oracle/) and the HIP
 * engine can be pinned bit-for-bit against the library the reference uses.
 *
 * Build + run: tests/golden/make_golden.sh (writes tests/golden/raw/, then
 * tests/golden/pack_golden.py packs it into tests/golden/mpich_golden.npz).
 *
 * Inputs: splitmix64 keyed by (case seed, rank, element index) — see gen().
 */
#include <mpi.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <stdint.h>
#include <math.h>
#include <complex.h>

static uint64_t splitmix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}
static uint64_t key(uint64_t seed, int rank, uint64_t i) {
    return splitmix64(seed * 0x100000001B3ull ^ ((uint64_t)rank << 40) ^ i);
}
/* uniform [-1,1) with 24 (f32) / 53 (f64) bits */
static float uf32(uint64_t r) { return (float)((int64_t)(r >> 40) - (1ll << 23)) / (float)(1 << 23); }
static double uf64(uint64_t r) { return (double)((int64_t)(r >> 11) - (1ll << 52)) / 4503599627370496.0; }

typedef struct { const char *name; MPI_Datatype dt; int esize; int kind; } DT;
/* kind: 0 signed int, 1 unsigned int, 2 f32, 3 f64, 4 c64, 5 c128, 6 byte */
static DT DTS[] = {
    {"INT8_T", MPI_INT8_T, 1, 0},     {"UINT8_T", MPI_UINT8_T, 1, 1},
    {"INT16_T", MPI_INT16_T, 2, 0},   {"UINT16_T", MPI_UINT16_T, 2, 1},
    {"INT32_T", MPI_INT32_T, 4, 0},   {"UINT32_T", MPI_UINT32_T, 4, 1},
    {"INT64_T", MPI_INT64_T, 8, 0},   {"UINT64_T", MPI_UINT64_T, 8, 1},
    {"BYTE", MPI_BYTE, 1, 6},         {"SHORT", MPI_SHORT, 2, 0},
    {"UNSIGNED_SHORT", MPI_UNSIGNED_SHORT, 2, 1},
    {"INT", MPI_INT, 4, 0},           {"UNSIGNED", MPI_UNSIGNED, 4, 1},
    {"LONG", MPI_LONG, 8, 0},         {"UNSIGNED_LONG", MPI_UNSIGNED_LONG, 8, 1},
    {"CHAR", MPI_CHAR, 1, 0},         {"SIGNED_CHAR", MPI_SIGNED_CHAR, 1, 0},
    {"UNSIGNED_CHAR", MPI_UNSIGNED_CHAR, 1, 1},
    {"WCHAR", MPI_WCHAR, 4, 0},
    {"FLOAT", MPI_FLOAT, 4, 2},       {"DOUBLE", MPI_DOUBLE, 8, 3},
    {"C_FLOAT_COMPLEX", MPI_C_FLOAT_COMPLEX, 8, 4},
    {"C_DOUBLE_COMPLEX", MPI_C_DOUBLE_COMPLEX, 16, 5},
};
#define NDT (int)(sizeof(DTS) / sizeof(DTS[0]))
typedef struct { const char *name; MPI_Op op; } OPD;
static OPD OPS[] = {
    {"SUM", MPI_SUM}, {"PROD", MPI_PROD}, {"MIN", MPI_MIN}, {"MAX", MPI_MAX},
    {"LAND", MPI_LAND}, {"LOR", MPI_LOR}, {"LXOR", MPI_LXOR},
    {"BAND", MPI_BAND}, {"BOR", MPI_BOR}, {"BXOR", MPI_BXOR},
};
#define NOP (int)(sizeof(OPS) / sizeof(OPS[0]))

static const DT *dt_by_name(const char *n) {
    for (int i = 0; i < NDT; i++) if (!strcmp(DTS[i].name, n)) return &DTS[i];
    abort();
}
static const OPD *op_by_name(const char *n) {
    for (int i = 0; i < NOP; i++) if (!strcmp(OPS[i].name, n)) return &OPS[i];
    abort();
}

/* gen modes */
enum { G_RAND = 0, G_LOGIC = 1, G_SMALL = 2, G_NAN = 3, G_SZERO = 4, G_RANKP1 = 5, G_EDGE = 6 };

/* fill `count` elements of rank `rank`'s buffer */
static void gen(void *buf, const DT *d, int count, int rank, int nranks, uint64_t seed, int mode) {
    unsigned char *b = (unsigned char *)buf;
    for (int i = 0; i < count; i++) {
        uint64_t r = key(seed, rank, (uint64_t)i);
        int zero = (mode == G_LOGIC) && ((r & 0xff) < 90);  /* ~35% zeros */
        unsigned char *e = b + (size_t)i * d->esize;
        switch (d->kind) {
        case 0: case 1: case 6: {
            uint64_t v = r;
            if (mode == G_SMALL) v = 1 + (r % 3);
            if (mode == G_RANKP1) v = (uint64_t)(rank + 1);
            if (mode == G_LOGIC && zero) v = 0;
            if (mode == G_EDGE) {
                /* extremes: 0, -1, min, max, 1 cycling by (rank+i) */
                int k = (rank + i) % 5;
                uint64_t mx = (d->kind == 0) ? ((1ull << (8 * d->esize - 1)) - 1) : (d->esize == 8 ? ~0ull : ((1ull << (8 * d->esize)) - 1));
                uint64_t mn = (d->kind == 0) ? (1ull << (8 * d->esize - 1)) : 0;
                v = k == 0 ? 0 : k == 1 ? ~0ull : k == 2 ? mn : k == 3 ? mx : 1;
            }
            memcpy(e, &v, d->esize); /* little endian: low bytes */
            break;
        }
        case 2: {
            float v = uf32(r);
            if (mode == G_SMALL) v = (float)(1 + (r % 3));
            if (mode == G_RANKP1) v = (float)(rank + 1);
            if (mode == G_LOGIC && zero) v = (r & 0x100) ? 0.0f : -0.0f;
            if (mode == G_NAN) { v = (float)(rank + 1) * (1 + i % 3); if (rank == (int)(seed % nranks) && (i % 2 == 0)) v = NAN; }
            if (mode == G_SZERO) v = (rank % 2) ? -0.0f : 0.0f;
            if (mode == G_EDGE) { int k = (rank + i) % 6; v = k == 0 ? INFINITY : k == 1 ? -INFINITY : k == 2 ? 1e-45f : k == 3 ? -0.0f : k == 4 ? 3.4e38f : uf32(r); }
            memcpy(e, &v, 4);
            break;
        }
        case 3: {
            double v = uf64(r);
            if (mode == G_SMALL) v = (double)(1 + (r % 3));
            if (mode == G_RANKP1) v = (double)(rank + 1);
            if (mode == G_LOGIC && zero) v = (r & 0x100) ? 0.0 : -0.0;
            if (mode == G_NAN) { v = (double)(rank + 1) * (1 + i % 3); if (rank == (int)(seed % nranks) && (i % 2 == 0)) v = NAN; }
            if (mode == G_SZERO) v = (rank % 2) ? -0.0 : 0.0;
            if (mode == G_EDGE) { int k = (rank + i) % 6; v = k == 0 ? INFINITY : k == 1 ? -INFINITY : k == 2 ? 5e-324 : k == 3 ? -0.0 : k == 4 ? 1.7e308 : uf64(r); }
            memcpy(e, &v, 8);
            break;
        }
        case 4: {
            float v[2] = {uf32(r), uf32(splitmix64(r))};
            if (mode == G_SMALL || mode == G_RANKP1) { v[0] = (float)(mode == G_RANKP1 ? rank + 1 : 1 + r % 3); v[1] = 0; }
            memcpy(e, v, 8);
            break;
        }
        case 5: {
            double v[2] = {uf64(r), uf64(splitmix64(r))};
            if (mode == G_SMALL || mode == G_RANKP1) { v[0] = (double)(mode == G_RANKP1 ? rank + 1 : 1 + r % 3); v[1] = 0; }
            memcpy(e, v, 16);
            break;
        }
        }
    }
}

static FILE *manifest;
static int g_rank, g_size;
static const char *outdir;
static int case_no = 0;

/* Gather `bytes` from every rank to rank 0 and write <outdir>/<id>.<tag>.bin */
static void dump(const char *id, const char *tag, const void *buf, size_t bytes) {
    unsigned char *all = NULL;
    if (g_rank == 0) all = malloc(bytes * g_size + 1);
    MPI_Gather(buf, (int)bytes, MPI_BYTE, all, (int)bytes, MPI_BYTE, 0, MPI_COMM_WORLD);
    if (g_rank == 0) {
        char path[512];
        snprintf(path, sizeof path, "%s/%s.%s.bin", outdir, id, tag);
        FILE *f = fopen(path, "wb");
        fwrite(all, 1, bytes * g_size, f);
        fclose(f);
        free(all);
    }
}

/* run one collective case */
static void run_case(const char *coll, const char *dtn, const char *opn, int count, int root, int mode, uint64_t seed) {
    const DT *d = dt_by_name(dtn);
    const OPD *o = opn ? op_by_name(opn) : NULL;
    int n = g_size;
    char id[256];
    snprintf(id, sizeof id, "n%d_%04d", n, case_no++);
    size_t in_elems = (size_t)count, out_elems = (size_t)count;
    if (!strcmp(coll, "allgather")) out_elems = (size_t)count * n;
    if (!strcmp(coll, "alltoall")) { in_elems = (size_t)count * n; out_elems = (size_t)count * n; }
    size_t ib = in_elems * d->esize, ob = out_elems * d->esize;
    unsigned char *in = calloc(ib + 16, 1), *out = malloc(ob + 16);
    gen(in, d, (int)in_elems, g_rank, n, seed, mode);
    memset(out, 0xCD, ob + 16); /* sentinel: shows "untouched" (Exscan rank 0, Reduce non-root) */
    int rc = MPI_SUCCESS;
    if (!strcmp(coll, "allreduce")) rc = MPI_Allreduce(in, out, count, d->dt, o->op, MPI_COMM_WORLD);
    else if (!strcmp(coll, "reduce")) rc = MPI_Reduce(in, out, count, d->dt, o->op, root, MPI_COMM_WORLD);
    else if (!strcmp(coll, "scan")) rc = MPI_Scan(in, out, count, d->dt, o->op, MPI_COMM_WORLD);
    else if (!strcmp(coll, "exscan")) rc = MPI_Exscan(in, out, count, d->dt, o->op, MPI_COMM_WORLD);
    else if (!strcmp(coll, "bcast")) { memcpy(out, in, ib); rc = MPI_Bcast(out, count, d->dt, root, MPI_COMM_WORLD); }
    else if (!strcmp(coll, "allgather")) rc = MPI_Allgather(in, count, d->dt, out, count, d->dt, MPI_COMM_WORLD);
    else if (!strcmp(coll, "alltoall")) rc = MPI_Alltoall(in, count, d->dt, out, count, d->dt, MPI_COMM_WORLD);
    else abort();
    dump(id, "in", in, ib);
    dump(id, "out", out, ob);
    if (g_rank == 0) {
        fprintf(manifest, "{\"id\":\"%s\",\"coll\":\"%s\",\"n\":%d,\"dtype\":\"%s\",\"op\":%s%s%s,\"count\":%d,\"root\":%d,\"mode\":%d,\"seed\":%llu,\"rc\":%d,\"in_bytes\":%zu,\"out_bytes\":%zu}\n",
                id, coll, n, dtn, o ? "\"" : "", o ? o->name : "null", o ? "\"" : "", count, root, mode,
                (unsigned long long)seed, rc, ib, ob);
        fflush(manifest);
    }
    free(in);
    free(out);
}

/* v-collectives: counts are a deterministic function of (seed, a, b) and may
 * be 0; displacements are packed (MPI.jl: disps = cumsum(counts) - counts,
 * collective.jl:169, :365, :425, :551-552).  Buffers are padded to the
 * largest rank's size so the dumps stay rectangular. */
static int vcnt(int seed, int a, int b, int base) { return ((a * 7 + b * 3 + seed) % 5) * base; }

static void run_vcase(const char *coll, const char *dtn, int base, int root, int seed) {
    const DT *d = dt_by_name(dtn);
    int n = g_size, r = g_rank;
    char id[256];
    snprintf(id, sizeof id, "n%d_%04d", n, case_no++);
    int cnt[16][16], sc[16], sd[16], rc_[16], rd[16];
    for (int a = 0; a < 16; a++)
        for (int b = 0; b < 16; b++) cnt[a][b] = vcnt(seed, a, b, base);
    size_t in_max = 0, out_max = 0, myin = 0, myout = 0;
    for (int q = 0; q < n; q++) {
        size_t i = 0, o = 0;
        if (!strcmp(coll, "gather")) { i = base; o = q == root ? (size_t)n * base : 0; }
        if (!strcmp(coll, "gatherv")) { i = cnt[q][0]; if (q == root) for (int p = 0; p < n; p++) o += cnt[p][0]; }
        if (!strcmp(coll, "scatter")) { i = q == root ? (size_t)n * base : 0; o = base; }
        if (!strcmp(coll, "scatterv")) { if (q == root) for (int p = 0; p < n; p++) i += cnt[p][1]; o = cnt[q][1]; }
        if (!strcmp(coll, "allgatherv")) { i = cnt[q][2]; for (int p = 0; p < n; p++) o += cnt[p][2]; }
        if (!strcmp(coll, "alltoallv")) { for (int p = 0; p < n; p++) { i += cnt[q][p]; o += cnt[p][q]; } }
        if (i > in_max) in_max = i;
        if (o > out_max) out_max = o;
        if (q == r) { myin = i; myout = o; }
    }
    size_t ib = in_max * d->esize + 16, ob = out_max * d->esize + 16;
    unsigned char *in = calloc(ib, 1), *out = malloc(ob);
    gen(in, d, (int)myin, r, n, seed, G_RAND);
    memset(out, 0xCD, ob);
    int rc = 0, acc = 0;
    if (!strcmp(coll, "gather")) rc = MPI_Gather(in, base, d->dt, out, base, d->dt, root, MPI_COMM_WORLD);
    else if (!strcmp(coll, "scatter")) rc = MPI_Scatter(in, base, d->dt, out, base, d->dt, root, MPI_COMM_WORLD);
    else if (!strcmp(coll, "gatherv")) {
        for (int p = 0; p < n; p++) { rc_[p] = cnt[p][0]; rd[p] = acc; acc += rc_[p]; }
        rc = MPI_Gatherv(in, cnt[r][0], d->dt, out, rc_, rd, d->dt, root, MPI_COMM_WORLD);
    } else if (!strcmp(coll, "scatterv")) {
        for (int p = 0; p < n; p++) { sc[p] = cnt[p][1]; sd[p] = acc; acc += sc[p]; }
        rc = MPI_Scatterv(in, sc, sd, d->dt, out, cnt[r][1], d->dt, root, MPI_COMM_WORLD);
    } else if (!strcmp(coll, "allgatherv")) {
        for (int p = 0; p < n; p++) { rc_[p] = cnt[p][2]; rd[p] = acc; acc += rc_[p]; }
        rc = MPI_Allgatherv(in, cnt[r][2], d->dt, out, rc_, rd, d->dt, MPI_COMM_WORLD);
    } else if (!strcmp(coll, "alltoallv")) {
        int a2 = 0;
        for (int p = 0; p < n; p++) { sc[p] = cnt[r][p]; sd[p] = acc; acc += sc[p]; rc_[p] = cnt[p][r]; rd[p] = a2; a2 += rc_[p]; }
        rc = MPI_Alltoallv(in, sc, sd, d->dt, out, rc_, rd, d->dt, MPI_COMM_WORLD);
    } else abort();
    dump(id, "in", in, ib);
    dump(id, "out", out, ob);
    if (g_rank == 0) {
        fprintf(manifest, "{\"id\":\"%s\",\"coll\":\"%s\",\"n\":%d,\"dtype\":\"%s\",\"op\":null,\"count\":%d,\"root\":%d,"
                "\"mode\":0,\"seed\":%d,\"rc\":%d,\"in_bytes\":%zu,\"out_bytes\":%zu,\"counts\":[",
                id, coll, n, dtn, base, root, seed, rc, ib, ob);
        for (int a = 0; a < n; a++) {
            fprintf(manifest, "%s[", a ? "," : "");
            for (int b = 0; b < n; b++) fprintf(manifest, "%s%d", b ? "," : "", cnt[a][b]);
            fprintf(manifest, "]");
        }
        fprintf(manifest, "]}\n");
        fflush(manifest);
    }
    free(in);
    free(out);
}

/* single-process probe of the op x type matrix and of the elementwise
 * semantics of MPI_Reduce_local(inbuf, inoutbuf) (mpi.h:1357) */
static void reduce_local_probe(void) {
    char path[512];
    snprintf(path, sizeof path, "%s/op_type_matrix.json", outdir);
    FILE *f = fopen(path, "w");
    fprintf(f, "{\n");
    int first = 1;
    for (int di = 0; di < NDT; di++) {
        for (int oi = 0; oi < NOP; oi++) {
            const DT *d = &DTS[di];
            const int count = 64;
            unsigned char a[64 * 16], b[64 * 16];
            int mode = (oi >= 4 && oi <= 6) ? G_LOGIC : G_EDGE;
            gen(a, d, count, 0, 2, 1000 + di * 16 + oi, mode);
            gen(b, d, count, 1, 2, 1000 + di * 16 + oi, mode);
            /* add a couple of random elements too */
            gen(a + 32 * d->esize, d, 32, 2, 3, 77 + di, mode == G_LOGIC ? G_LOGIC : G_RAND);
            gen(b + 32 * d->esize, d, 32, 3, 4, 78 + di, mode == G_LOGIC ? G_LOGIC : G_RAND);
            unsigned char inout[64 * 16];
            memcpy(inout, b, count * d->esize);
            int rc = MPI_Reduce_local(a, inout, count, d->dt, OPS[oi].op);
            int cls = rc;
            MPI_Error_class(rc, &cls);
            fprintf(f, "%s  \"%s/%s\": %d", first ? "" : ",\n", d->name, OPS[oi].name, cls);
            first = 0;
            if (rc == MPI_SUCCESS) {
                char id[128];
                snprintf(id, sizeof id, "local_%s_%s", d->name, OPS[oi].name);
                snprintf(path, sizeof path, "%s/%s.in.bin", outdir, id);
                FILE *g = fopen(path, "wb"); fwrite(a, 1, count * d->esize, g); fwrite(b, 1, count * d->esize, g); fclose(g);
                snprintf(path, sizeof path, "%s/%s.out.bin", outdir, id);
                g = fopen(path, "wb"); fwrite(inout, 1, count * d->esize, g); fclose(g);
                fprintf(manifest, "{\"id\":\"%s\",\"coll\":\"reduce_local\",\"n\":2,\"dtype\":\"%s\",\"op\":\"%s\",\"count\":%d,\"root\":0,\"mode\":%d,\"seed\":0,\"rc\":0,\"in_bytes\":%d,\"out_bytes\":%d}\n",
                        id, d->name, OPS[oi].name, count, mode, count * d->esize, count * d->esize);
            }
        }
    }
    fprintf(f, "\n}\n");
    fclose(f);
}

int main(int argc, char **argv) {
    MPI_Init(&argc, &argv);
    MPI_Comm_rank(MPI_COMM_WORLD, &g_rank);
    MPI_Comm_size(MPI_COMM_WORLD, &g_size);
    MPI_Comm_set_errhandler(MPI_COMM_WORLD, MPI_ERRORS_RETURN);
    outdir = argc > 1 ? argv[1] : ".";
    if (g_rank == 0) {
        char path[512];
        snprintf(path, sizeof path, "%s/manifest_n%d.jsonl", outdir, g_size);
        manifest = fopen(path, "w");
    }
    if (g_size == 1) {
        reduce_local_probe();
    } else {
        int n = g_size;
        /* --- Allreduce: association (float SUM/PROD) below & above the 2048 B
         *     recursive-doubling threshold, ints, logic, NaN/±0 edges --- */
        const int counts_f[] = {1, 5, 64, 600, 1100};
        for (int c = 0; c < 5; c++) {
            run_case("allreduce", "FLOAT", "SUM", counts_f[c], 0, G_RAND, 11 + c);
            run_case("allreduce", "DOUBLE", "SUM", counts_f[c], 0, G_RAND, 21 + c);
        }
        run_case("allreduce", "FLOAT", "PROD", 600, 0, G_RAND, 31);
        run_case("allreduce", "DOUBLE", "PROD", 64, 0, G_RAND, 32);
        run_case("allreduce", "C_FLOAT_COMPLEX", "SUM", 300, 0, G_RAND, 33);
        run_case("allreduce", "C_DOUBLE_COMPLEX", "PROD", 40, 0, G_RAND, 34);
        run_case("allreduce", "FLOAT", "MAX", 600, 0, G_RAND, 35);
        run_case("allreduce", "DOUBLE", "MIN", 100, 0, G_RAND, 36);
        run_case("allreduce", "FLOAT", "LAND", 64, 0, G_LOGIC, 37);
        run_case("allreduce", "DOUBLE", "LXOR", 64, 0, G_LOGIC, 38);
        const char *ints[] = {"INT8_T", "UINT8_T", "INT16_T", "UINT16_T", "INT32_T", "UINT32_T", "INT64_T", "UINT64_T"};
        const char *iops[] = {"SUM", "PROD", "MIN", "MAX", "LAND", "LOR", "LXOR", "BAND", "BOR", "BXOR"};
        for (int t = 0; t < 8; t++)
            for (int o = 0; o < 10; o++)
                run_case("allreduce", ints[t], iops[o], o < 2 ? 300 : 33, 0, (o >= 4 && o <= 6) ? G_LOGIC : G_RAND, 100 + t * 10 + o);
        run_case("allreduce", "INT8_T", "SUM", 8, 0, G_SMALL, 201);
        run_case("allreduce", "INT8_T", "PROD", 8, 0, G_RANKP1, 202);
        /* NaN / signed-zero edges (pin operand rule of MPIR MIN/MAX) */
        for (int s = 0; s < n; s++) {
            run_case("allreduce", "FLOAT", "MAX", 16, 0, G_NAN, (uint64_t)s);
            run_case("allreduce", "FLOAT", "MIN", 16, 0, G_NAN, (uint64_t)(s + n));
        }
        run_case("allreduce", "FLOAT", "MAX", 16, 0, G_SZERO, 5);
        run_case("allreduce", "FLOAT", "MIN", 16, 0, G_SZERO, 6);
        run_case("allreduce", "DOUBLE", "MAX", 16, 0, G_SZERO, 7);
        run_case("allreduce", "FLOAT", "SUM", 1024, 0, G_SZERO, 8);
        /* reference test shapes (test/test_allreduce.jl:24-55): Int64 1:len */
        run_case("allreduce", "INT64_T", "SUM", 27, 0, G_RANKP1, 9);
        /* --- Reduce (root n-1 as test_reduce.jl:18, and root 0) --- */
        run_case("reduce", "FLOAT", "SUM", 600, n - 1, G_RAND, 301);
        run_case("reduce", "FLOAT", "SUM", 64, 0, G_RAND, 302);
        run_case("reduce", "DOUBLE", "SUM", 1100, 0, G_RAND, 303);
        run_case("reduce", "INT32_T", "BAND", 1000, n - 1, G_RAND, 304);
        run_case("reduce", "INT64_T", "BOR", 1000, 0, G_RAND, 305);
        run_case("reduce", "INT32_T", "MAX", 1000, n / 2, G_RAND, 306);
        run_case("reduce", "INT64_T", "MAX", 100, n - 1, G_RAND, 307);
        run_case("reduce", "FLOAT", "MAX", 16, n - 1, G_NAN, 1);
        /* --- Scan / Exscan (recursive doubling association) --- */
        const char *sdt[] = {"FLOAT", "DOUBLE", "INT32_T", "INT64_T"};
        for (int t = 0; t < 4; t++) {
            run_case("scan", sdt[t], "SUM", t < 2 ? 700 : 100, 0, G_RAND, 401 + t);
            run_case("exscan", sdt[t], "SUM", t < 2 ? 700 : 100, 0, G_RAND, 411 + t);
            run_case("scan", sdt[t], "PROD", 4, 0, G_RANKP1, 421 + t);
            run_case("exscan", sdt[t], "PROD", 4, 0, G_RANKP1, 431 + t);
        }
        const char *bops[] = {"BAND", "BOR", "MAX"};
        for (int o = 0; o < 3; o++) {
            run_case("scan", "INT32_T", bops[o], 512, 0, G_RAND, 441 + o);
            run_case("exscan", "INT32_T", bops[o], 512, 0, G_RAND, 451 + o);
            run_case("scan", "INT64_T", bops[o], 512, 0, G_RAND, 461 + o);
            run_case("exscan", "INT64_T", bops[o], 512, 0, G_RAND, 471 + o);
        }
        run_case("scan", "FLOAT", "MAX", 16, 0, G_NAN, 2);
        run_case("exscan", "FLOAT", "MIN", 16, 0, G_NAN, 3);
        /* --- Bcast / Allgather / Alltoall (bit copies) --- */
        run_case("bcast", "FLOAT", NULL, 289, 0, G_RAND, 501);
        run_case("bcast", "INT8_T", NULL, 1001, n - 1, G_RAND, 502);
        run_case("allgather", "FLOAT", NULL, 1, 0, G_RANKP1, 503);
        run_case("allgather", "C_DOUBLE_COMPLEX", NULL, 37, 0, G_RAND, 504);
        run_case("alltoall", "FLOAT", NULL, 1, 0, G_RANKP1, 505);
        run_case("alltoall", "INT16_T", NULL, 129, 0, G_RAND, 506);
        /* --- v-collectives / rooted variants --- */
        const char *vcolls[] = {"gather", "gatherv", "scatter", "scatterv", "allgatherv", "alltoallv"};
        for (int v = 0; v < 6; v++) {
            run_vcase(vcolls[v], "FLOAT", 1, 0, 601 + v);
            run_vcase(vcolls[v], "INT8_T", 37, n - 1, 611 + v);
            run_vcase(vcolls[v], "C_DOUBLE_COMPLEX", 29, n / 2, 621 + v);
        }
    }
    if (g_rank == 0) fclose(manifest);
    MPI_Finalize();
    return 0;
}
