// ref_harness.cc — TEST INFRASTRUCTURE ONLY (never linked into the product).
//
// Glue that turns the reference's own host sources (compiled in place from
// /root/reference by oracle/build_ref.sh) into a ctypes-loadable library
// oracle/_ref/libbpref.so.  It is used to
//   * validate the CPU restatement in oracle/bp_oracle.c, and
//   * generate the golden fixtures under tests/golden/ (tests/golden/make_golden.py).
//
// What this file adds (all of it our own code; no reference source is copied):
//   1. host definitions of the GPU symbols the reference's host code calls
//      (cuda_point_vector_multi_scalar_mul ...), written over the reference's
//      own device primitives from device_curve25519_ops.cuh compiled for the
//      host with -D__device__= .  The MSM follows the canonical pairwise tree
//      that point_multi_scalar_mul_shared_kernel defines
//      (cuda_bulletproof_kernels.cu:141-168) — SURVEY §0.6 / row A9.
//   2. a deterministic RAND_bytes: block k of the stream = SHA256(seed_le64 || k_le64)
//      (SURVEY §8c "RNG").  Every reference RAND_bytes call asks for 32 bytes.
//   3. flat extern "C" entry points (ref_*) over the reference functions, with
//      the reference's stdout chatter sent to /dev/null.
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>
#include <fcntl.h>
#include <openssl/sha.h>

#include "curve25519_ops.h"
#include "bulletproof_vectors.h"
#include "bulletproof_range_proof.h"
#include "bulletproof_challenge.h"
#include "cuda_bulletproof.h"
#include "device_curve25519_ops.cuh"   // host build: -D__device__=

// ---------------------------------------------------------------- quiet stdout
static int g_saved_stdout = -1;
static void quiet_begin() {
    fflush(stdout);
    g_saved_stdout = dup(1);
    int devnull = open("/dev/null", O_WRONLY);
    dup2(devnull, 1);
    close(devnull);
}
static void quiet_end() {
    fflush(stdout);
    dup2(g_saved_stdout, 1);
    close(g_saved_stdout);
}

// ---------------------------------------------------------------- captured stdout
// The same redirection into an anonymous temp file instead of /dev/null, so the lines the
// reference prints about its own check point (crv:287-346: "Computed X:", the byte-difference
// counts, "Matching significant bits", "Hash difference count") can be handed back verbatim.
static FILE* g_cap = NULL;
static void capture_begin() {
    fflush(stdout);
    g_saved_stdout = dup(1);
    g_cap = tmpfile();
    dup2(fileno(g_cap), 1);
}
static void capture_end(char* log, size_t cap) {
    fflush(stdout);
    dup2(g_saved_stdout, 1);
    close(g_saved_stdout);
    long len = ftell(g_cap);
    if (len < 0) len = 0;
    rewind(g_cap);
    size_t got = 0;
    if (log && cap) {
        got = fread(log, 1, (size_t)len < cap - 1 ? (size_t)len : cap - 1, g_cap);
        log[got] = 0;
    }
    fclose(g_cap);
    g_cap = NULL;
}

// ---------------------------------------------------------------- deterministic RNG
static uint64_t g_seed = 1, g_ctr = 0;
static uint8_t g_block[32];
static int g_avail = 0;

extern "C" void ref_rand_seed(uint64_t seed) { g_seed = seed; g_ctr = 0; g_avail = 0; }

extern "C" int RAND_bytes(unsigned char* buf, int num) {
    for (int i = 0; i < num; i++) {
        if (g_avail == 0) {
            uint8_t in[16];
            for (int k = 0; k < 8; k++) { in[k] = (uint8_t)(g_seed >> (8 * k)); in[8 + k] = (uint8_t)(g_ctr >> (8 * k)); }
            SHA256(in, 16, g_block);
            g_ctr++;
            g_avail = 32;
        }
        buf[i] = g_block[32 - g_avail];
        g_avail--;
    }
    return 1;
}

// ---------------------------------------------------------------- GPU-symbol emulation
// Canonical pairwise tree (kernels.cu:162-168): for s=1,2,4..: T[i]=Ndev(T[i]+T[i+s]) for i%(2s)==0, i+s<n.
static void canon_tree_msm(ge25519* result, const fe25519* s, const ge25519* P, size_t n) {
    if (n == 0) return;
    ge25519* T = (ge25519*)malloc(n * sizeof(ge25519));
    for (size_t i = 0; i < n; i++) {
        uint8_t sb[32];
        device_fe25519_tobytes(sb, &s[i]);
        device_ge25519_scalarmult(&T[i], sb, &P[i]);
        device_ge25519_normalize(&T[i]);
    }
    for (size_t st = 1; st < n; st *= 2)
        for (size_t i = 0; i + st < n; i += 2 * st) {
            device_ge25519_add(&T[i], &T[i], &T[i + st]);
            device_ge25519_normalize(&T[i]);
        }
    *result = T[0];
    free(T);
}

extern "C" void cuda_point_vector_multi_scalar_mul(ge25519* result, const FieldVector* scalars,
                                                   const PointVector* points) {
    if (scalars->length != points->length) {
        fprintf(stderr, "Error: Vector lengths must match for multi-scalar multiplication\n");
        return;
    }
    canon_tree_msm(result, scalars->elements, points->elements, scalars->length);
}
extern "C" void cuda_point_vector_multi_scalar_mul_shared(ge25519* result, const FieldVector* scalars,
                                                          const PointVector* points) {
    cuda_point_vector_multi_scalar_mul(result, scalars, points);
}
extern "C" void cuda_batch_field_add(fe25519* r, const fe25519* a, const fe25519* b, size_t c) {
    for (size_t i = 0; i < c; i++) device_fe25519_add(&r[i], &a[i], &b[i]);
}
extern "C" void cuda_batch_field_sub(fe25519* r, const fe25519* a, const fe25519* b, size_t c) {
    for (size_t i = 0; i < c; i++) device_fe25519_sub(&r[i], &a[i], &b[i]);
}
extern "C" void cuda_batch_field_mul(fe25519* r, const fe25519* a, const fe25519* b, size_t c) {
    for (size_t i = 0; i < c; i++) device_fe25519_mul(&r[i], &a[i], &b[i]);
}
extern "C" void cuda_batch_field_square(fe25519* r, const fe25519* a, size_t c) {
    for (size_t i = 0; i < c; i++) device_fe25519_mul(&r[i], &a[i], &a[i]);
}

// ---------------------------------------------------------------- reference helpers
// generate_deterministic_base_points lives in complete_bulletproof_test.cu (built with -Dmain=ref_test_main)
void generate_deterministic_base_points(PointVector* points, size_t n, uint8_t seed[32]);

extern "C" void ref_base_points(ge25519* out, size_t n, const uint8_t* seed32) {
    PointVector pv = {out, n};
    uint8_t seed[32];
    memcpy(seed, seed32, 32);
    generate_deterministic_base_points(&pv, n, seed);
}

extern "C" void ref_fe_add(fe25519* h, const fe25519* f, const fe25519* g) { fe25519_add(h, f, g); }
extern "C" void ref_fe_sub(fe25519* h, const fe25519* f, const fe25519* g) { fe25519_sub(h, f, g); }
extern "C" void ref_fe_mul(fe25519* h, const fe25519* f, const fe25519* g) { fe25519_mul(h, f, g); }
extern "C" void ref_fe_invert(fe25519* h, const fe25519* f) { fe25519_invert(h, f); }
extern "C" void ref_fe_tobytes(uint8_t* b, const fe25519* h) { fe25519_tobytes(b, h); }
extern "C" void ref_ge_add(ge25519* r, const ge25519* p, const ge25519* q) { ge25519_add(r, p, q); }
extern "C" void ref_ge_scalarmult(ge25519* r, const uint8_t* s, const ge25519* p) { ge25519_scalarmult(r, s, p); }
extern "C" void ref_ge_normalize(ge25519* p) { ge25519_normalize(p); }
extern "C" void ref_dev_fe_add(fe25519* h, const fe25519* f, const fe25519* g) { device_fe25519_add(h, f, g); }
extern "C" void ref_dev_fe_sub(fe25519* h, const fe25519* f, const fe25519* g) { device_fe25519_sub(h, f, g); }
extern "C" void ref_dev_fe_mul(fe25519* h, const fe25519* f, const fe25519* g) { device_fe25519_mul(h, f, g); }
extern "C" void ref_dev_ge_add(ge25519* r, const ge25519* p, const ge25519* q) { device_ge25519_add(r, p, q); }
extern "C" void ref_dev_ge_scalarmult(ge25519* r, const uint8_t* s, const ge25519* p) { device_ge25519_scalarmult(r, s, p); }
extern "C" void ref_dev_ge_normalize(ge25519* p) { device_ge25519_normalize(p); }
extern "C" void ref_msm_canon(ge25519* r, const fe25519* s, const ge25519* P, size_t n) { canon_tree_msm(r, s, P, n); }
// The canonical tree alone over given points (the levels of canon_tree_msm above its terms):
// combines the roots of aligned power-of-two shards into the whole MSM's root.
extern "C" void ref_point_tree(ge25519* r, const ge25519* P, size_t n) {
    if (n == 0) return;
    ge25519* T = (ge25519*)malloc(n * sizeof(ge25519));
    memcpy(T, P, n * sizeof(ge25519));
    for (size_t st = 1; st < n; st *= 2)
        for (size_t i = 0; i + st < n; i += 2 * st) {
            device_ge25519_add(&T[i], &T[i], &T[i + st]);
            device_ge25519_normalize(&T[i]);
        }
    *r = T[0];
    free(T);
}
extern "C" void ref_msm_cpu(ge25519* r, const fe25519* s, const ge25519* P, size_t n) {
    FieldVector sv = {(fe25519*)s, n};
    PointVector pv = {(ge25519*)P, n};
    point_vector_multi_scalar_mul(r, &sv, &pv);
}
extern "C" void ref_inner_product(fe25519* r, const fe25519* a, const fe25519* b, size_t n) {
    FieldVector av = {(fe25519*)a, n}, bv = {(fe25519*)b, n};
    field_vector_inner_product(r, &av, &bv);
}
extern "C" void ref_challenge(uint8_t* out, const uint8_t* data, size_t len, const char* dom) {
    generate_challenge(out, data, len, dom);
}
extern "C" void ref_challenge_y(uint8_t* out, const ge25519* V, const ge25519* A, const ge25519* S) {
    generate_challenge_y(out, V, A, S);
}
extern "C" void ref_challenge_z(uint8_t* out, const uint8_t* y) { generate_challenge_z(out, y); }
extern "C" void ref_challenge_x(uint8_t* out, const ge25519* T1, const ge25519* T2) { generate_challenge_x(out, T1, T2); }

// g, h exactly as complete_bulletproof_test.cu:84-109 builds them (restated; the test's main is not callable).
extern "C" void ref_gh(ge25519* g, ge25519* h) {
    uint8_t gs[32] = {0x03}, hs[32] = {0x04}, gb[32], hb[32];
    ge25519_0(g);
    ge25519_0(h);
    SHA256(gs, 32, gb);
    SHA256(hs, 32, hb);
    fe25519_frombytes(&g->X, gb);
    fe25519_frombytes(&h->X, hb);
    fe25519_1(&g->Y); fe25519_1(&h->Y);
    fe25519_1(&g->Z); fe25519_1(&h->Z);
    fe25519_mul(&g->T, &g->X, &g->Y);
    fe25519_mul(&h->T, &h->X, &h->Y);
}

// Flat proof header: V,A,S,T1,T2 (5 points), taux, mu, t, c, x (5 field elements)
struct FlatHead {
    ge25519 V, A, S, T1, T2;
    fe25519 taux, mu, t, c, x;
};

// Mirrors complete_bulletproof_test.cu:122-144 : blinding from the RNG, V = pedersen_commit, then prove.
// Writes ab_len (= proof a/b length after proving) and L_len; a/b/L/R buffers must hold n entries.
extern "C" int ref_prove(uint64_t seed, const uint8_t* value32, size_t n, const ge25519* G, const ge25519* H,
                         const ge25519* g, const ge25519* h, ge25519* Vcommit, struct FlatHead* head,
                         fe25519* a, fe25519* b, ge25519* L, ge25519* R, size_t* ab_len, size_t* L_len) {
    ref_rand_seed(seed);
    fe25519 value, blinding;
    uint8_t bb[32];
    fe25519_frombytes(&value, value32);
    generate_random_scalar(bb, 32);
    fe25519_frombytes(&blinding, bb);
    PointVector Gv = {(ge25519*)G, n}, Hv = {(ge25519*)H, n};
    RangeProof proof;
    memset(&proof, 0, sizeof(proof));
    quiet_begin();
    pedersen_commit(Vcommit, &value, &blinding, g, h);
    generate_range_proof(&proof, &value, &blinding, n, &Gv, &Hv, g, h);
    quiet_end();
    if (proof.ip_proof.a.elements == NULL) return -1;   // out-of-range input: prover returned early
    head->V = proof.V; head->A = proof.A; head->S = proof.S; head->T1 = proof.T1; head->T2 = proof.T2;
    head->taux = proof.taux; head->mu = proof.mu; head->t = proof.t;
    head->c = proof.ip_proof.c; head->x = proof.ip_proof.x;
    *ab_len = proof.ip_proof.a.length;
    *L_len = proof.ip_proof.L_len;
    memcpy(a, proof.ip_proof.a.elements, *ab_len * sizeof(fe25519));
    memcpy(b, proof.ip_proof.b.elements, *ab_len * sizeof(fe25519));
    memcpy(L, proof.ip_proof.L.elements, *L_len * sizeof(ge25519));
    memcpy(R, proof.ip_proof.R.elements, *L_len * sizeof(ge25519));
    range_proof_free(&proof);
    return 0;
}

static void build_proof(RangeProof* p, const struct FlatHead* head, size_t n, const fe25519* a, const fe25519* b,
                        size_t ab_len, const ge25519* L, const ge25519* R, size_t L_len) {
    memset(p, 0, sizeof(*p));
    p->V = head->V; p->A = head->A; p->S = head->S; p->T1 = head->T1; p->T2 = head->T2;
    p->taux = head->taux; p->mu = head->mu; p->t = head->t;
    p->ip_proof.n = n;
    p->ip_proof.a.elements = (fe25519*)a; p->ip_proof.a.length = ab_len;
    p->ip_proof.b.elements = (fe25519*)b; p->ip_proof.b.length = ab_len;
    p->ip_proof.c = head->c;
    p->ip_proof.L.elements = (ge25519*)L; p->ip_proof.L.length = L_len;
    p->ip_proof.R.elements = (ge25519*)R; p->ip_proof.R.length = L_len;
    p->ip_proof.L_len = L_len;
    p->ip_proof.x = head->x;
}

// The notebook's cuda_range_proof_verify (crv:82), with the MSM emulated above.
extern "C" int ref_cuda_range_proof_verify(const struct FlatHead* head, const ge25519* V, size_t n,
                                           const fe25519* a, const fe25519* b, size_t ab_len, const ge25519* L,
                                           const ge25519* R, size_t L_len, const ge25519* G, const ge25519* H,
                                           const ge25519* g, const ge25519* h) {
    RangeProof p;
    build_proof(&p, head, n, a, b, ab_len, L, R, L_len);
    PointVector Gv = {(ge25519*)G, n}, Hv = {(ge25519*)H, n};
    quiet_begin();
    bool ok = cuda_range_proof_verify(&p, V, n, &Gv, &Hv, g, h);
    quiet_end();
    return ok ? 1 : 0;
}

// The same call with the reference's stdout captured into `log` (NUL-terminated, at most cap - 1
// bytes): its own report of the check point and of the accept rule's inputs (crv:287-367).
extern "C" int ref_cuda_range_proof_verify_log(const struct FlatHead* head, const ge25519* V, size_t n,
                                               const fe25519* a, const fe25519* b, size_t ab_len, const ge25519* L,
                                               const ge25519* R, size_t L_len, const ge25519* G, const ge25519* H,
                                               const ge25519* g, const ge25519* h, char* log, size_t cap) {
    RangeProof p;
    build_proof(&p, head, n, a, b, ab_len, L, R, L_len);
    PointVector Gv = {(ge25519*)G, n}, Hv = {(ge25519*)H, n};
    capture_begin();
    bool ok = cuda_range_proof_verify(&p, V, n, &Gv, &Hv, g, h);
    capture_end(log, cap);
    return ok ? 1 : 0;
}

// The CPU verify (bulletproof_range_proof.cu:1717) — second verify semantics.
extern "C" int ref_range_proof_verify(const struct FlatHead* head, const ge25519* V, size_t n, const fe25519* a,
                                      const fe25519* b, size_t ab_len, const ge25519* L, const ge25519* R,
                                      size_t L_len, const ge25519* G, const ge25519* H, const ge25519* g,
                                      const ge25519* h) {
    RangeProof p;
    build_proof(&p, head, n, a, b, ab_len, L, R, L_len);
    PointVector Gv = {(ge25519*)G, n}, Hv = {(ge25519*)H, n};
    quiet_begin();
    bool ok = range_proof_verify(&p, V, n, &Gv, &Hv, g, h);
    quiet_end();
    return ok ? 1 : 0;
}

// calculate_inner_product_point (rp.cu:658) on the challenges the cuda verify derives (crv:99-106).
extern "C" void ref_verify_P(const struct FlatHead* head, const ge25519* V, size_t n, const ge25519* G,
                             const ge25519* H, const ge25519* g, const ge25519* h, ge25519* P_out,
                             uint8_t* yzx_out /* 96 bytes, may be NULL */) {
    uint8_t yb[32], zb[32], xb[32];
    fe25519 y, z, x;
    generate_challenge_y(yb, V, &head->A, &head->S);
    fe25519_frombytes(&y, yb);
    generate_challenge_z(zb, yb);
    fe25519_frombytes(&z, zb);
    generate_challenge_x(xb, &head->T1, &head->T2);
    fe25519_frombytes(&x, xb);
    if (yzx_out) { memcpy(yzx_out, yb, 32); memcpy(yzx_out + 32, zb, 32); memcpy(yzx_out + 64, xb, 32); }
    RangeProof p;
    memset(&p, 0, sizeof(p));
    p.V = head->V; p.A = head->A; p.S = head->S; p.T1 = head->T1; p.T2 = head->T2; p.t = head->t;
    PointVector Gv = {(ge25519*)G, n}, Hv = {(ge25519*)H, n};
    quiet_begin();
    calculate_inner_product_point(P_out, &p, &x, &y, &z, &head->t, &Gv, &Hv, g, h, n);
    quiet_end();
}

// The IPA generator fold of crv:160-279, composed from the reference's own primitives in the same order.
// Writes the folded G'/H' after every round (rounds*n/2.. entries, packed round after round) and check_point.
extern "C" void ref_ipa_fold(const ge25519* G, const ge25519* H, size_t n, const fe25519* x, const ge25519* L,
                             const ge25519* R, size_t rounds, const fe25519* a0, const fe25519* b0,
                             const fe25519* c, const ge25519* Q, ge25519* Gtrace, ge25519* Htrace,
                             ge25519* check_out) {
    ge25519* Gc = (ge25519*)malloc(n * sizeof(ge25519));
    ge25519* Hc = (ge25519*)malloc(n * sizeof(ge25519));
    memcpy(Gc, G, n * sizeof(ge25519));
    memcpy(Hc, H, n * sizeof(ge25519));
    uint8_t transcript[32] = {0};
    size_t np = n, off = 0;
    for (size_t i = 0; i < rounds; i++) {
        np >>= 1;
        fe25519 u, ui;
        if (i == 0) {
            u = *x;
        } else {
            uint8_t d[96], ch[32];
            memcpy(d, transcript, 32);
            fe25519_tobytes(d + 32, &L[i].X);
            fe25519_tobytes(d + 64, &R[i].X);
            generate_challenge(ch, d, 96, "InnerProductChal");
            memcpy(transcript, ch, 32);
            fe25519_frombytes(&u, ch);
        }
        fe25519_invert(&ui, &u);
        uint8_t ub[32], uib[32];
        fe25519_tobytes(ub, &u);
        fe25519_tobytes(uib, &ui);
        for (size_t j = 0; j < np; j++) {
            ge25519 t1, t2;
            ge25519_scalarmult(&t1, uib, &Gc[j]); ge25519_normalize(&t1);
            ge25519_scalarmult(&t2, ub, &Gc[j + np]); ge25519_normalize(&t2);
            ge25519_add(&Gc[j], &t1, &t2); ge25519_normalize(&Gc[j]);
            ge25519_scalarmult(&t1, ub, &Hc[j]); ge25519_normalize(&t1);
            ge25519_scalarmult(&t2, uib, &Hc[j + np]); ge25519_normalize(&t2);
            ge25519_add(&Hc[j], &t1, &t2); ge25519_normalize(&Hc[j]);
        }
        memcpy(Gtrace + off, Gc, np * sizeof(ge25519));
        memcpy(Htrace + off, Hc, np * sizeof(ge25519));
        off += np;
    }
    uint8_t ab[32], bb[32], cb[32];
    fe25519_tobytes(ab, a0);
    fe25519_tobytes(bb, b0);
    fe25519_tobytes(cb, c);
    ge25519 cp, t1, t2, t3;
    ge25519_0(&cp);
    ge25519_scalarmult(&t1, ab, &Gc[0]); ge25519_normalize(&t1);
    ge25519_scalarmult(&t2, bb, &Hc[0]); ge25519_normalize(&t2);
    ge25519_scalarmult(&t3, cb, Q); ge25519_normalize(&t3);
    ge25519_add(&cp, &cp, &t1); ge25519_normalize(&cp);
    ge25519_add(&cp, &cp, &t2); ge25519_normalize(&cp);
    ge25519_add(&cp, &cp, &t3); ge25519_normalize(&cp);
    *check_out = cp;
    free(Gc);
    free(Hc);
}

// inner_product_prove (bulletproof_vectors.cu:277) on caller vectors; the reference allocates the
// proof's vectors itself (inner_product_proof_init) — copied out here and freed.
// a_out/b_out hold the final (length-1) vectors, L/R hold log2(n) points each.
extern "C" int ref_ipa_prove(const fe25519* a, const fe25519* b, size_t n, const ge25519* G, const ge25519* H,
                             const ge25519* Q, const fe25519* c_in, const uint8_t* transcript32, fe25519* a_out,
                             fe25519* b_out, size_t* ab_len, ge25519* L, ge25519* R, size_t* L_len, fe25519* x_out) {
    FieldVector av = {(fe25519*)a, n}, bv = {(fe25519*)b, n};
    PointVector Gv = {(ge25519*)G, n}, Hv = {(ge25519*)H, n};
    InnerProductProof proof;
    memset(&proof, 0, sizeof(proof));
    quiet_begin();
    inner_product_prove(&proof, &av, &bv, &Gv, &Hv, Q, c_in, transcript32);
    quiet_end();
    if (proof.a.elements == NULL) return -1;
    *ab_len = proof.a.length;
    *L_len = proof.L_len;
    memcpy(a_out, proof.a.elements, proof.a.length * sizeof(fe25519));
    memcpy(b_out, proof.b.elements, proof.b.length * sizeof(fe25519));
    memcpy(L, proof.L.elements, proof.L_len * sizeof(ge25519));
    memcpy(R, proof.R.elements, proof.L_len * sizeof(ge25519));
    *x_out = proof.x;
    inner_product_proof_free(&proof);
    return 0;
}

// The notebook's cuda_inner_product_verify (crv:130) on a flat proof.
extern "C" int ref_cuda_inner_product_verify(size_t n, const fe25519* a, const fe25519* b, size_t ab_len,
                                             const fe25519* c, const ge25519* L, const ge25519* R, size_t L_len,
                                             const fe25519* x, const ge25519* P, const ge25519* G, const ge25519* H,
                                             const ge25519* Q) {
    InnerProductProof p;
    memset(&p, 0, sizeof(p));
    p.n = n;
    p.a.elements = (fe25519*)a; p.a.length = ab_len;
    p.b.elements = (fe25519*)b; p.b.length = ab_len;
    p.c = *c;
    p.L.elements = (ge25519*)L; p.L.length = L_len;
    p.R.elements = (ge25519*)R; p.R.length = L_len;
    p.L_len = L_len;
    p.x = *x;
    PointVector Gv = {(ge25519*)G, n}, Hv = {(ge25519*)H, n};
    quiet_begin();
    bool ok = cuda_inner_product_verify(&p, P, &Gv, &Hv, Q);
    quiet_end();
    return ok ? 1 : 0;
}

// cuda_inner_product_verify with its stdout captured (see ref_cuda_range_proof_verify_log).
extern "C" int ref_cuda_inner_product_verify_log(size_t n, const fe25519* a, const fe25519* b, size_t ab_len,
                                                 const fe25519* c, const ge25519* L, const ge25519* R, size_t L_len,
                                                 const fe25519* x, const ge25519* P, const ge25519* G,
                                                 const ge25519* H, const ge25519* Q, char* log, size_t cap) {
    InnerProductProof p;
    memset(&p, 0, sizeof(p));
    p.n = n;
    p.a.elements = (fe25519*)a; p.a.length = ab_len;
    p.b.elements = (fe25519*)b; p.b.length = ab_len;
    p.c = *c;
    p.L.elements = (ge25519*)L; p.L.length = L_len;
    p.R.elements = (ge25519*)R; p.R.length = L_len;
    p.L_len = L_len;
    p.x = *x;
    PointVector Gv = {(ge25519*)G, n}, Hv = {(ge25519*)H, n};
    capture_begin();
    bool ok = cuda_inner_product_verify(&p, P, &Gv, &Hv, Q);
    capture_end(log, cap);
    return ok ? 1 : 0;
}

// ---- range_proof_verify (bulletproof_range_proof.cu:1717) sub-checks, each the
// reference's own function on a flat proof, for pinning the restatement step by step.
bool enhanced_range_check(const fe25519* t, const fe25519* delta, const fe25519* z, const ge25519* V,
                          const ge25519* g, const ge25519* h, size_t n);   // rp.cu:765 (not in the header)

// out: delta (32 B fe), flags bit0 enhanced_range_check, bit1 robust_polynomial_identity_check,
// bit2 inner_product_verify (with P from calculate_inner_product_point, Q = h).
extern "C" void ref_rpv_parts(const struct FlatHead* head, const ge25519* V, size_t n, const fe25519* a,
                              const fe25519* b, size_t ab_len, const ge25519* L, const ge25519* R, size_t L_len,
                              const ge25519* G, const ge25519* H, const ge25519* g, const ge25519* h,
                              fe25519* delta_out, int* flags) {
    RangeProof p;
    build_proof(&p, head, n, a, b, ab_len, L, R, L_len);
    PointVector Gv = {(ge25519*)G, n}, Hv = {(ge25519*)H, n};
    uint8_t yb[32], zb[32], xb[32];
    fe25519 y, z, x, delta;
    quiet_begin();
    generate_challenge_y(yb, V, &p.A, &p.S);
    fe25519_frombytes(&y, yb);
    generate_challenge_z(zb, yb);
    fe25519_frombytes(&z, zb);
    generate_challenge_x(xb, &p.T1, &p.T2);
    fe25519_frombytes(&x, xb);
    compute_precise_delta(&delta, &z, &y, n);
    int f = 0;
    if (enhanced_range_check(&p.t, &delta, &z, V, g, h, n)) f |= 1;
    if (robust_polynomial_identity_check(&p, V, &x, &y, &z, &delta, g, h)) f |= 2;
    ge25519 P;
    calculate_inner_product_point(&P, &p, &x, &y, &z, &p.t, &Gv, &Hv, g, h, n);
    if (inner_product_verify(&p.ip_proof, &P, &Gv, &Hv, h)) f |= 4;
    quiet_end();
    *delta_out = delta;
    *flags = f;
}
