/* sanitize_driver.c — TEST INFRASTRUCTURE (tests/test_sanitizers.py): drives the CPU restatement
 * (oracle/bp_oracle.c) through its whole surface under AddressSanitizer + UndefinedBehaviour-
 * Sanitizer: field/point primitives on edge limbs, MSMs (canonical, CPU order, Pippenger), the
 * inner products, SHA-256, a prove -> verify round trip at n = 16 in all three verify semantics.
 * Prints "ok <accepts>" and exits 0; a sanitizer report aborts with a non-zero status. */
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include "../oracle/bp_oracle.h"

static uint64_t st = 0x9E3779B97F4A7C15ull;
static uint64_t rnd(void) {
    st ^= st << 13;
    st ^= st >> 7;
    st ^= st << 17;
    return st;
}

int main(void) {
    enum { N = 16, M = 37 };
    const uint64_t E[] = {0, 1, 19, 0xFFFFFFFFFFFFFFEDull, 0xFFFFFFFFFFFFFFFFull, 0x7FFFFFFFFFFFFFFFull,
                          0x79435E50D79435E5ull};
    orc_fe f[M], g[M], r[M];
    for (int i = 0; i < M; i++)
        for (int k = 0; k < 4; k++) {
            f[i].v[k] = (i % 3 == 0) ? E[rnd() % 7] : rnd();
            g[i].v[k] = (i % 5 == 0) ? E[rnd() % 7] : rnd();
        }
    uint8_t bytes[32];
    for (int i = 0; i < M; i++) {
        orc_fe_add(&r[i], &f[i], &g[i]);
        orc_fe_sub(&r[i], &r[i], &g[i]);
        orc_fe_mul(&r[i], &r[i], &f[i]);
        orc_fe_invert(&r[i], &r[i]);
        orc_fe_square_kernel(&r[i], &r[i]);
        orc_fe_tobytes(bytes, &r[i]);
    }
    orc_ge P[M], q, t;
    uint8_t seed[32] = {5};
    orc_base_points(P, M, seed);
    orc_ge_zero(&q);
    for (int i = 0; i < 4; i++) {
        orc_ge_add(&q, &q, &P[i]);
        orc_ge_scalarmult(&t, bytes, &P[i]);
        orc_ge_normalize_host(&t);
        orc_ge_normalize_dev(&t);
    }
    orc_msm_canon(&t, f, P, M);
    orc_point_tree(&t, P, M);
    orc_msm_cpu(&t, f, P, 5);
    orc_msm_pippenger(&t, f, P, M, 4);
    orc_msm_pippenger(&t, f, P, 1, 12);
    orc_inner_product(&r[0], f, g, M);
    orc_ip_gpu(&r[0], f, g, M);
    orc_ip_gpu_shared(&r[0], f, g, 16);
    orc_ip_gpu_batch(r, f, g, 6, 3);
    orc_sha256(bytes, (const uint8_t*)"abc", 3);
    orc_challenge(bytes, (const uint8_t*)"abc", 3, "y_ch");
    /* prove -> verify, n = 16, value 42 (complete_bulletproof_test.cu:116) */
    orc_ge G[N], H[N], gg, hh;
    uint8_t s1[32] = {1}, s2[32] = {2};
    orc_base_points(G, N, s1);
    orc_base_points(H, N, s2);
    orc_gh(&gg, &hh);
    int accepts = 0;
    for (int trial = 0; trial < 3; trial++) {
        uint8_t value[32] = {0}, gamma[32], sLR[2 * N * 32], r4[4][32];
        value[0] = (uint8_t)(42 + trial);
        for (int i = 0; i < 32; i++) gamma[i] = (uint8_t)rnd();
        for (int i = 0; i < 2 * N * 32; i++) sLR[i] = (uint8_t)rnd();
        for (int k = 0; k < 4; k++)
            for (int i = 0; i < 32; i++) r4[k][i] = (uint8_t)rnd();
        orc_head head;
        orc_fe a[1], b[1];
        orc_ge L[4], R[4], Pout, chk, Gt[N], Ht[N];
        size_t Llen = 0;
        if (orc_generate_range_proof(value, gamma, sLR, (const uint8_t(*)[32])r4, N, G, H, &gg, &hh, &head, a, b, L,
                                     R, &Llen) != 0)
            return 2;
        accepts += orc_cuda_range_proof_verify(&head, &head.V, N, a, b, 1, L, R, Llen, G, H, &gg, &hh, &Pout, &chk,
                                               Gt, Ht);
        accepts += orc_cuda_inner_product_verify(N, a, b, 1, &head.c, L, R, Llen, &head.x, &Pout, G, H, &hh, &chk,
                                                 Gt, Ht);
        orc_rpv_detail det;
        accepts += orc_range_proof_verify(&head, &head.V, N, a, b, 1, L, R, Llen, G, H, &gg, &hh, &det);
    }
    printf("ok %d\n", accepts);
    return 0;
}
