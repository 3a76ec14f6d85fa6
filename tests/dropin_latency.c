/* dropin_latency.c — wall-clock latency of the drop-in cuda_range_proof_verify (cuda_bulletproof.h:61)
 * as the reference's own caller sees it: one proof per call, host structs, through
 * libcudabulletproof_hip.so.  Built by tests/test_dropin.py and bench.py's configs0 leg:
 *
 *   gcc -O2 -I include tests/dropin_latency.c -L cudabulletproof_amd -lcudabulletproof_hip -o <bin>
 *   <bin> proof.bin [warm_calls]
 *
 * proof.bin (little-endian): u64 n, ab_len, L_len; G[n], H[n], g, h, V (ge25519, 128 B each);
 * head: A, S, T1, T2 (ge25519), taux, mu, t, c, x (fe25519); a[ab_len], b[ab_len]; L[L_len], R[L_len].
 *
 * Prints one JSON line: process start -> first call (the library's constructors and nothing else),
 * the HIP runtime's own start-up (hipbp_device_count, the first HIP call), the first verify (engine
 * and pipeline set-up, code-object loads, the verify), and the median / min of the warm calls; all
 * CLOCK_MONOTONIC wall time (the reference driver's clock() at complete_bulletproof_test.cu:150-157
 * is process CPU time).  Exit status 0 when every call returned the same verdict. */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "cudabulletproof_hip.h"

static double now_ms(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec * 1e3 + ts.tv_nsec * 1e-6;
}

static int cmp_d(const void* a, const void* b) {
    double x = *(const double*)a, y = *(const double*)b;
    return x < y ? -1 : x > y;
}

static void* rd(FILE* f, size_t bytes) {
    void* p = malloc(bytes ? bytes : 1);
    if (!p || fread(p, 1, bytes, f) != bytes) {
        fprintf(stderr, "dropin_latency: short read\n");
        exit(2);
    }
    return p;
}

int main(int argc, char** argv) {
    double t_start = now_ms();
    if (argc < 2) {
        fprintf(stderr, "usage: %s proof.bin [warm_calls]\n", argv[0]);
        return 2;
    }
    int warm = argc > 2 ? atoi(argv[2]) : 20;
    if (warm < 1 || warm > 10000) warm = 20;
    FILE* f = fopen(argv[1], "rb");
    if (!f) {
        perror(argv[1]);
        return 2;
    }
    uint64_t hdr[3];
    if (fread(hdr, 8, 3, f) != 3) return 2;
    size_t n = hdr[0], abl = hdr[1], Lr = hdr[2];
    ge25519* G = rd(f, n * sizeof(ge25519));
    ge25519* H = rd(f, n * sizeof(ge25519));
    ge25519* gh = rd(f, 3 * sizeof(ge25519));   /* g, h, V */
    RangeProof rp;
    memset(&rp, 0, sizeof rp);
    if (fread(&rp.A, sizeof(ge25519), 4, f) != 4 || fread(&rp.taux, sizeof(fe25519), 3, f) != 3 ||
        fread(&rp.ip_proof.c, sizeof(fe25519), 1, f) != 1 || fread(&rp.ip_proof.x, sizeof(fe25519), 1, f) != 1)
        return 2;
    rp.V = gh[2];
    rp.ip_proof.n = n;
    rp.ip_proof.a.elements = rd(f, abl * sizeof(fe25519));
    rp.ip_proof.a.length = abl;
    rp.ip_proof.b.elements = rd(f, abl * sizeof(fe25519));
    rp.ip_proof.b.length = abl;
    rp.ip_proof.L.elements = rd(f, Lr * sizeof(ge25519));
    rp.ip_proof.L.length = Lr;
    rp.ip_proof.R.elements = rd(f, Lr * sizeof(ge25519));
    rp.ip_proof.R.length = Lr;
    rp.ip_proof.L_len = Lr;
    fclose(f);
    PointVector Gv = {G, n}, Hv = {H, n};

    double t0 = now_ms();
    int ndev = hipbp_device_count();   /* the HIP runtime's own start-up */
    double t1 = now_ms();
    bool first = cuda_range_proof_verify(&rp, &gh[2], n, &Gv, &Hv, &gh[0], &gh[1]);
    double t2 = now_ms();
    double* w = malloc(warm * sizeof(double));
    int same = 1;
    for (int i = 0; i < warm; i++) {
        double a = now_ms();
        bool ok = cuda_range_proof_verify(&rp, &gh[2], n, &Gv, &Hv, &gh[0], &gh[1]);
        w[i] = now_ms() - a;
        same &= ok == first;
    }
    qsort(w, warm, sizeof(double), cmp_d);
    printf("{\"n\": %zu, \"devices\": %d, \"verdict\": %s, \"same_verdict_every_call\": %s, "
           "\"to_first_call_ms\": %.3f, \"runtime_init_ms\": %.3f, \"first_call_ms\": %.3f, "
           "\"first_call_incl_runtime_init_ms\": %.3f, \"warm_median_ms\": %.3f, \"warm_min_ms\": %.3f, "
           "\"warm_calls\": %d}\n",
           n, ndev, first ? "true" : "false", same ? "true" : "false", t0 - t_start, t1 - t0, t2 - t1, t2 - t0,
           w[warm / 2], w[0], warm);
    return same ? 0 : 1;
}
