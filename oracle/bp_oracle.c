/* bp_oracle.c — TEST INFRASTRUCTURE ONLY (see bp_oracle.h).
 *
 * A plain-C restatement of the reference's arithmetic and of the verify path
 * it runs through cuda_bulletproof.h, written from the semantics in SURVEY
 * Appendix B, quirks included (lossy borrow chains, truncated 19x fold,
 * 13-step "invert", k = d in the point add, host vs device normalize).
 * Every function cites the reference file:line it restates.
 */
#include "bp_oracle.h"
#include <stdlib.h>
#include <string.h>

/* curve25519_ops.cu:7-8 */
static const uint64_t PRIME[4] = {0xFFFFFFFFFFFFFFEDull, 0xFFFFFFFFFFFFFFFFull, 0xFFFFFFFFFFFFFFFFull,
                                  0x7FFFFFFFFFFFFFFFull};
/* curve25519_ops.cu:341-346 — the constant used as "2d" (it is d) */
static const uint8_t KBYTES[32] = {0xA3, 0x78, 0x59, 0x13, 0xCA, 0x4D, 0xEB, 0x75, 0xAB, 0xD8, 0x41,
                                   0x41, 0x4D, 0x0A, 0x70, 0x00, 0x98, 0xE8, 0x79, 0x77, 0x79, 0x40,
                                   0xC7, 0x8C, 0x73, 0xFE, 0x6F, 0x2B, 0xEE, 0x6C, 0x03, 0x52};

/* ------------------------------------------------------------------ SHA-256 (FIPS 180-4) */
static const uint32_t SHA_K[64] = {
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
    0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
    0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
    0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
    0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
    0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
    0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
    0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};

#define ROR(x, n) (((x) >> (n)) | ((x) << (32 - (n))))

static void sha_block(uint32_t st[8], const uint8_t* p) {
    uint32_t w[64];
    for (int i = 0; i < 16; i++)
        w[i] = ((uint32_t)p[4 * i] << 24) | ((uint32_t)p[4 * i + 1] << 16) | ((uint32_t)p[4 * i + 2] << 8) | p[4 * i + 3];
    for (int i = 16; i < 64; i++) {
        uint32_t s0 = ROR(w[i - 15], 7) ^ ROR(w[i - 15], 18) ^ (w[i - 15] >> 3);
        uint32_t s1 = ROR(w[i - 2], 17) ^ ROR(w[i - 2], 19) ^ (w[i - 2] >> 10);
        w[i] = w[i - 16] + s0 + w[i - 7] + s1;
    }
    uint32_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4], f = st[5], g = st[6], h = st[7];
    for (int i = 0; i < 64; i++) {
        uint32_t t1 = h + (ROR(e, 6) ^ ROR(e, 11) ^ ROR(e, 25)) + ((e & f) ^ (~e & g)) + SHA_K[i] + w[i];
        uint32_t t2 = (ROR(a, 2) ^ ROR(a, 13) ^ ROR(a, 22)) + ((a & b) ^ (a & c) ^ (b & c));
        h = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
    }
    st[0] += a; st[1] += b; st[2] += c; st[3] += d; st[4] += e; st[5] += f; st[6] += g; st[7] += h;
}

typedef struct { uint32_t st[8]; uint8_t buf[64]; size_t used; uint64_t total; } sha_ctx;

static void sha_init(sha_ctx* c) {
    static const uint32_t iv[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a,
                                   0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
    memcpy(c->st, iv, sizeof iv);
    c->used = 0;
    c->total = 0;
}
static void sha_update(sha_ctx* c, const uint8_t* d, size_t n) {
    c->total += n;
    while (n) {
        size_t k = 64 - c->used;
        if (k > n) k = n;
        memcpy(c->buf + c->used, d, k);
        c->used += k; d += k; n -= k;
        if (c->used == 64) { sha_block(c->st, c->buf); c->used = 0; }
    }
}
static void sha_final(sha_ctx* c, uint8_t out[32]) {
    uint64_t bits = c->total * 8;
    uint8_t pad = 0x80, zero = 0;
    sha_update(c, &pad, 1);
    while (c->used != 56) sha_update(c, &zero, 1);
    uint8_t lenb[8];
    for (int i = 0; i < 8; i++) lenb[i] = (uint8_t)(bits >> (56 - 8 * i));
    sha_update(c, lenb, 8);
    for (int i = 0; i < 8; i++) {
        out[4 * i] = (uint8_t)(c->st[i] >> 24); out[4 * i + 1] = (uint8_t)(c->st[i] >> 16);
        out[4 * i + 2] = (uint8_t)(c->st[i] >> 8); out[4 * i + 3] = (uint8_t)c->st[i];
    }
}
void orc_sha256(uint8_t out[32], const uint8_t* data, size_t len) {
    sha_ctx c;
    sha_init(&c);
    sha_update(&c, data, len);
    sha_final(&c, out);
}

/* bulletproof_challenge.cu:6-21 : SHA256(domain || data), clear bit 255 */
void orc_challenge(uint8_t out[32], const uint8_t* data, size_t len, const char* dom) {
    sha_ctx c;
    sha_init(&c);
    sha_update(&c, (const uint8_t*)dom, strlen(dom));
    sha_update(&c, data, len);
    sha_final(&c, out);
    out[31] &= 0x7F;
}

/* ------------------------------------------------------------------ field */
static void fe_from_le(orc_fe* h, const uint8_t* b) { /* curve25519_ops.cu:254 */
    for (int i = 0; i < 4; i++) {
        uint64_t v = 0;
        for (int k = 7; k >= 0; k--) v = (v << 8) | b[8 * i + k];
        h->v[i] = v;
    }
}
static void fe_to_le_raw(uint8_t* b, const orc_fe* h) { /* device_curve25519_ops.cuh:33 */
    for (int i = 0; i < 4; i++)
        for (int k = 0; k < 8; k++) b[8 * i + k] = (uint8_t)(h->v[i] >> (8 * k));
}
static int ge_prime(const uint64_t t[4]) { /* the ">= p" test of curve25519_ops.cu:54-59 */
    for (int i = 3; i >= 0; i--) {
        if (t[i] > PRIME[i]) return 1;
        if (t[i] < PRIME[i]) return 0;
    }
    return 1;
}
/* LOSSYSUB: borrow = h < lo64(p_i + borrow) — drops the borrow when p_i + 1 wraps */
static void lossy_sub_p(uint64_t t[4]) {
    uint64_t br = 0;
    for (int i = 0; i < 4; i++) {
        uint64_t pb = PRIME[i] + br;
        uint64_t d = t[i] - PRIME[i] - br;
        br = t[i] < pb;
        t[i] = d;
    }
}
/* curve25519_ops.cu:41-68 : exact 257-bit sum, then one lossy "-p" */
void orc_fe_add(orc_fe* h, const orc_fe* f, const orc_fe* g) {
    uint64_t t[4];
    unsigned __int128 acc = 0;
    for (int i = 0; i < 4; i++) {
        acc += (unsigned __int128)f->v[i] + g->v[i];
        t[i] = (uint64_t)acc;
        acc >>= 64;
    }
    if (acc || ge_prime(t)) lossy_sub_p(t);
    memcpy(h->v, t, sizeof t);
}
/* curve25519_ops.cu:71-90 : lossy borrow chain, then lossy "+p" */
void orc_fe_sub(orc_fe* h, const orc_fe* f, const orc_fe* g) {
    uint64_t t[4], br = 0;
    for (int i = 0; i < 4; i++) {
        uint64_t gb = g->v[i] + br;
        t[i] = f->v[i] - g->v[i] - br;
        br = f->v[i] < gb;
    }
    if (br) {
        uint64_t cy = 0;
        for (int i = 0; i < 4; i++) {
            t[i] += PRIME[i] + cy;
            cy = t[i] < PRIME[i];
        }
    }
    memcpy(h->v, t, sizeof t);
}
/* fold of the 512-bit product t[0..7] (curve25519_ops.cu:114-145) */
static void fold512(orc_fe* h, uint64_t t[8]) {
    uint64_t c = t[4] * 19;
    t[0] += c;
    uint64_t cy = t[0] < c;
    for (int i = 1; i < 4; i++) {
        c = t[i + 4] * 19 + cy;
        t[i] += c;
        cy = t[i] < c;
    }
    if (cy || ge_prime(t)) lossy_sub_p(t);
    memcpy(h->v, t, 4 * sizeof(uint64_t));
}
/* curve25519_ops.cu:93-146 : exact 512-bit schoolbook product + quirky fold */
void orc_fe_mul(orc_fe* h, const orc_fe* f, const orc_fe* g) {
    uint64_t t[8] = {0};
    for (int i = 0; i < 4; i++) {
        uint64_t carry = 0;
        for (int j = 0; j < 4; j++) {
            unsigned __int128 m = (unsigned __int128)f->v[i] * g->v[j] + t[i + j] + carry;
            t[i + j] = (uint64_t)m;
            carry = (uint64_t)(m >> 64);
        }
        t[i + 4] = carry;
    }
    fold512(h, t);
}
/* cuda_field_ops.cu:147-216 field_square_kernel: carries between limbs are dropped and
 * 2*a_i*a_j is taken mod 2^128 — a different function from fe25519_sq. */
void orc_fe_square_kernel(orc_fe* h, const orc_fe* f) {
    uint64_t t[8] = {0};
    for (int i = 0; i < 4; i++) {
        unsigned __int128 d = (unsigned __int128)f->v[i] * f->v[i];
        t[2 * i] += (uint64_t)d;
        if (2 * i + 1 < 8) t[2 * i + 1] += (uint64_t)(d >> 64);
        for (int j = i + 1; j < 4; j++) {
            unsigned __int128 m = 2 * ((unsigned __int128)f->v[i] * f->v[j]);
            t[i + j] += (uint64_t)m;
            if (i + j + 1 < 8) t[i + j + 1] += (uint64_t)(m >> 64);
        }
    }
    fold512(h, t);
}
/* curve25519_ops.cu:157-207 : the fixed 13-multiplication chain (not an inverse) */
void orc_fe_invert(orc_fe* h, const orc_fe* f) {
    orc_fe t0, t1, t2;
    orc_fe_mul(&t0, f, f);
    orc_fe_mul(&t1, &t0, &t0);
    orc_fe_mul(&t1, &t1, &t1);
    orc_fe_mul(&t1, &t1, f);
    orc_fe_mul(&t0, &t1, &t0);
    orc_fe_mul(&t1, &t0, &t0);
    orc_fe_mul(&t1, &t1, &t1);
    orc_fe_mul(&t1, &t1, &t1);
    orc_fe_mul(&t1, &t1, &t1);
    orc_fe_mul(&t1, &t1, &t1);
    orc_fe_mul(&t2, f, f);
    orc_fe_mul(&t2, &t2, f);
    orc_fe_mul(&t1, &t1, &t2);
    *h = t1;
}
/* curve25519_ops.cu:220-251 : one lossy conditional "-p", then LE bytes */
void orc_fe_tobytes(uint8_t* out, const orc_fe* h) {
    orc_fe t = *h;
    if (ge_prime(t.v)) lossy_sub_p(t.v);
    fe_to_le_raw(out, &t);
}
static void fe_set(orc_fe* h, uint64_t v) { h->v[0] = v; h->v[1] = h->v[2] = h->v[3] = 0; }

/* ------------------------------------------------------------------ points */
void orc_ge_zero(orc_ge* h) { /* curve25519_ops.cu:318 */
    fe_set(&h->X, 0); fe_set(&h->Y, 1); fe_set(&h->Z, 1); fe_set(&h->T, 0);
}
/* curve25519_ops.cu:326-378 (device copy: device_curve25519_ops.cuh:188-241) */
void orc_ge_add(orc_ge* r, const orc_ge* p, const orc_ge* q) {
    orc_fe A, B, C, D, E, F, G, H, k, t;
    orc_fe_sub(&A, &p->Y, &p->X);
    orc_fe_sub(&t, &q->Y, &q->X);
    orc_fe_mul(&A, &A, &t);
    orc_fe_add(&B, &p->Y, &p->X);
    orc_fe_add(&t, &q->Y, &q->X);
    orc_fe_mul(&B, &B, &t);
    fe_from_le(&k, KBYTES);
    orc_fe_mul(&C, &p->T, &q->T);
    orc_fe_mul(&C, &C, &k);
    orc_fe_mul(&D, &p->Z, &q->Z);
    orc_fe_add(&D, &D, &D);
    orc_fe_sub(&E, &B, &A);
    orc_fe_sub(&F, &D, &C);
    orc_fe_add(&G, &D, &C);
    orc_fe_add(&H, &B, &A);
    orc_fe_mul(&r->X, &E, &F);
    orc_fe_mul(&r->Y, &G, &H);
    orc_fe_mul(&r->Z, &F, &G);
    orc_fe_mul(&r->T, &E, &H);
}
/* curve25519_ops.cu:397-415 (== device_curve25519_ops.cuh:272-290): MSB-first double-and-add, all 256 bits */
void orc_ge_scalarmult(orc_ge* r, const uint8_t* s, const orc_ge* p) {
    orc_ge acc;
    orc_ge_zero(&acc);
    for (int i = 255; i >= 0; i--) {
        orc_ge_add(&acc, &acc, &acc);
        if ((s[i / 8] >> (i % 8)) & 1) orc_ge_add(&acc, &acc, p);
    }
    *r = acc;
}
/* curve25519_ops.cu:574-605 : early exit when canonical bytes of Z are 1, else the "invert" chain */
void orc_ge_normalize_host(orc_ge* p) {
    uint8_t zb[32];
    static const uint8_t one[32] = {1};
    orc_fe_tobytes(zb, &p->Z);
    if (memcmp(zb, one, 32) == 0) return;
    orc_fe zi, x, y, t;
    orc_fe_invert(&zi, &p->Z);
    orc_fe_mul(&x, &p->X, &zi);
    orc_fe_mul(&y, &p->Y, &zi);
    orc_fe_mul(&t, &x, &y);
    p->X = x; p->Y = y; fe_set(&p->Z, 1); p->T = t;
}
/* device_curve25519_ops.cuh:243-270 : z_inv hard-coded to 1 */
void orc_ge_normalize_dev(orc_ge* p) {
    orc_fe one;
    fe_set(&one, 1);
    orc_fe_mul(&p->X, &p->X, &one);
    orc_fe_mul(&p->Y, &p->Y, &one);
    fe_set(&p->Z, 1);
    orc_fe_mul(&p->T, &p->X, &p->Y);
}

/* ------------------------------------------------------------------ MSM / inner product */
/* cuda_bulletproof_kernels.cu:26-42 + canonical tree of :162-168 */
void orc_msm_canon(orc_ge* r, const orc_fe* s, const orc_ge* P, size_t n) {
    if (n == 0) return;
    orc_ge* T = (orc_ge*)malloc(n * sizeof(orc_ge));
    for (size_t i = 0; i < n; i++) {
        uint8_t sb[32];
        fe_to_le_raw(sb, &s[i]);
        orc_ge_scalarmult(&T[i], sb, &P[i]);
        orc_ge_normalize_dev(&T[i]);
    }
    orc_point_tree(r, T, n);
    free(T);
}
/* the reduction half of the GPU MSM: canonical pairwise tree, device normalize at each node
 * (cuda_bulletproof_kernels.cu:45-58 / :162-168).  P is not modified. */
void orc_point_tree(orc_ge* r, const orc_ge* P, size_t n) {
    if (n == 0) return;
    orc_ge* T = (orc_ge*)malloc(n * sizeof(orc_ge));
    memcpy(T, P, n * sizeof(orc_ge));
    for (size_t st = 1; st < n; st *= 2)
        for (size_t i = 0; i + st < n; i += 2 * st) {
            orc_ge_add(&T[i], &T[i], &T[i + st]);
            orc_ge_normalize_dev(&T[i]);
        }
    *r = T[0];
    free(T);
}
/* Pippenger with c-bit windows (4 <= c <= 16), W = ceil(256/c) windows, NB = 2^c buckets,
 * chunks of M = 16 buckets.  No normalization anywhere; Id = ge25519_0 (curve25519_ops.cu:318);
 * add = ge25519_add; smul = ge25519_scalarmult on the scalar's raw LE bytes.
 *   digit_w(i) = bits [c w, c w + c) of s_i (raw limbs)
 *   B_{w,b}  = pairwise tree over the points with digit b, in index order (level s = 1, 2, 4, ...:
 *              T[j] = add(T[j], T[j+s]) for j % 2s == 0, j + s < len); Id when the bucket is empty
 *   chunk k of window w (buckets kM .. kM+M-1): R = S = B_{kM+M-1}; for j = M-2 .. 1:
 *              R = add(R, B_{kM+j}); S = add(S, R); then R = add(R, B_{kM});
 *              V_{w,k} = add(S, smul(kM, R))
 *   S_w      = pairwise tree over V_{w,0..NB/M-1}
 *   T = S_{W-1}; for w = W-2 .. 0: c times T = add(T, T); T = add(T, S_w).  Result T. */
static void tree_inplace(orc_ge* T, size_t n) {
    for (size_t st = 1; st < n; st *= 2)
        for (size_t i = 0; i + st < n; i += 2 * st) orc_ge_add(&T[i], &T[i], &T[i + st]);
}
/* Window sums Sw[w0 .. w1) of the bucket MSM (a multi-GPU Pippenger splits the windows over the
 * ranks: each rank forms its windows' sums, the ranks exchange them, every rank runs the Horner). */
void orc_pippenger_windows(orc_ge* Sw, const orc_fe* s, const orc_ge* P, size_t n, int c, int w0, int w1) {
    const int M = 16;
    const size_t NB = (size_t)1 << c, NC = NB / M;
    orc_ge* Bk = (orc_ge*)malloc(NB * sizeof(orc_ge));
    orc_ge* V = (orc_ge*)malloc(NC * sizeof(orc_ge));
    orc_ge* tmp = (orc_ge*)malloc((n ? n : 1) * sizeof(orc_ge));
    uint32_t* dig = (uint32_t*)malloc((n ? n : 1) * sizeof(uint32_t));
    size_t* cnt = (size_t*)malloc((NB + 1) * sizeof(size_t));
    size_t* pos = (size_t*)malloc(NB * sizeof(size_t));
    for (int w = w0; w < w1; w++) {
        for (size_t i = 0; i < n; i++) {
            int lo = c * w;
            uint32_t d = 0;
            for (int b = 0; b < c && lo + b < 256; b++)
                d |= (uint32_t)((s[i].v[(lo + b) >> 6] >> ((lo + b) & 63)) & 1) << b;
            dig[i] = d;
        }
        /* stable counting sort of the points by digit: each bucket's points in index order */
        memset(cnt, 0, (NB + 1) * sizeof(size_t));
        for (size_t i = 0; i < n; i++) cnt[dig[i] + 1]++;
        for (size_t b = 0; b < NB; b++) cnt[b + 1] += cnt[b];
        memcpy(pos, cnt, NB * sizeof(size_t));
        for (size_t i = 0; i < n; i++) tmp[pos[dig[i]]++] = P[i];
        for (size_t b = 0; b < NB; b++) {
            size_t len = cnt[b + 1] - cnt[b];
            if (!len) { orc_ge_zero(&Bk[b]); continue; }
            tree_inplace(tmp + cnt[b], len);
            Bk[b] = tmp[cnt[b]];
        }
        for (size_t k = 0; k < NC; k++) {
            const orc_ge* Bc = Bk + k * M;
            orc_ge R = Bc[M - 1], S = Bc[M - 1], sm;
            for (int j = M - 2; j >= 1; j--) {
                orc_ge_add(&R, &R, &Bc[j]);
                orc_ge_add(&S, &S, &R);
            }
            orc_ge_add(&R, &R, &Bc[0]);
            uint8_t kb[32] = {0};
            uint64_t km = (uint64_t)k * M;
            for (int b = 0; b < 8; b++) kb[b] = (uint8_t)(km >> (8 * b));
            orc_ge_scalarmult(&sm, kb, &R);
            orc_ge_add(&V[k], &S, &sm);
        }
        tree_inplace(V, NC);
        Sw[w] = V[0];
    }
    free(Bk); free(V); free(tmp); free(dig); free(cnt); free(pos);
}

/* Horner over all W = ceil(256 / c) window sums, top window first: c doublings, then + S_w. */
void orc_pippenger_horner(orc_ge* r, const orc_ge* Sw, int c) {
    const int W = (256 + c - 1) / c;
    orc_ge T = Sw[W - 1];
    for (int w = W - 2; w >= 0; w--) {
        for (int d = 0; d < c; d++) orc_ge_add(&T, &T, &T);
        orc_ge_add(&T, &T, &Sw[w]);
    }
    *r = T;
}

void orc_msm_pippenger(orc_ge* r, const orc_fe* s, const orc_ge* P, size_t n, int c) {
    const int W = (256 + c - 1) / c;
    orc_ge* Sw = (orc_ge*)malloc(W * sizeof(orc_ge));
    orc_pippenger_windows(Sw, s, P, n, c, 0, W);
    orc_pippenger_horner(r, Sw, c);
    free(Sw);
}

/* bulletproof_vectors.cu:189-224 : sequential, host bytes and host normalize */
void orc_msm_cpu(orc_ge* r, const orc_fe* s, const orc_ge* P, size_t n) {
    orc_ge acc;
    orc_ge_zero(&acc);
    for (size_t i = 0; i < n; i++) {
        uint8_t sb[32];
        orc_ge t;
        orc_fe_tobytes(sb, &s[i]);
        orc_ge_scalarmult(&t, sb, &P[i]);
        orc_ge_normalize_host(&t);
        if (i == 0) {
            acc = t;
        } else {
            orc_ge_add(&acc, &acc, &t);
            orc_ge_normalize_host(&acc);
        }
    }
    orc_ge_normalize_host(&acc);
    *r = acc;
}
/* bulletproof_vectors.cu:101-114 : sequential left fold */
void orc_inner_product(orc_fe* r, const orc_fe* a, const orc_fe* b, size_t n) {
    orc_fe acc, t;
    fe_set(&acc, 0);
    for (size_t i = 0; i < n; i++) {
        orc_fe_mul(&t, &a[i], &b[i]);
        orc_fe_add(&acc, &acc, &t);
    }
    *r = acc;
}

/* cuda_inner_product.cu:154-183 + :185-216: one block of nt = min(n,512) threads; products for
 * t < nt, then halving tree from nt/2 with t + stride < n (elements >= nt are never read). */
void orc_ip_gpu_shared(orc_fe* r, const orc_fe* a, const orc_fe* b, size_t n) {
    size_t nt = n < 512 ? n : 512;
    if (nt == 0) return;
    orc_fe* s = (orc_fe*)malloc(nt * sizeof(orc_fe));
    for (size_t t = 0; t < nt; t++) orc_fe_mul(&s[t], &a[t], &b[t]);
    for (size_t st = nt / 2; st > 0; st >>= 1)
        for (size_t t = 0; t < st; t++)
            if (t + st < n) orc_fe_add(&s[t], &s[t], &s[t + st]);
    *r = s[0];
    free(s);
}
/* one 256-thread block of field_vector_inner_product_kernel (cuda_inner_product.cu:33-61) /
 * batch_inner_product_kernel (:260-299, warp_tail): grid-stride fold from 0, tree over 256 slots */
static void ip_block(orc_fe* out, const orc_fe* a, const orc_fe* b, size_t n, size_t blk, size_t grid_threads,
                     int warp_tail) {
    orc_fe s[256];
    for (size_t t = 0; t < 256; t++) {
        orc_fe acc, p;
        fe_set(&acc, 0);
        for (size_t idx = blk * 256 + t; idx < n; idx += grid_threads) {
            orc_fe_mul(&p, &a[idx], &b[idx]);
            orc_fe_add(&acc, &acc, &p);
        }
        s[t] = acc;
    }
    size_t stop = warp_tail ? 32 : 1;
    for (size_t st = 128; st >= stop; st >>= 1)
        for (size_t t = 0; t < st; t++) orc_fe_add(&s[t], &s[t], &s[t + st]);
    if (warp_tail)
        for (size_t st = 16; st >= 1; st >>= 1)
            for (size_t t = 0; t < st; t++) orc_fe_add(&s[t], &s[t], &s[t + st]);
    *out = s[0];
}
/* cuda_inner_product.cu:97-151: n <= 512 -> shared form; else grid of min(ceil(n/256),1024)
 * blocks, then fe25519_reduce_kernel (:69-92) over at most 256 partials. */
void orc_ip_gpu(orc_fe* r, const orc_fe* a, const orc_fe* b, size_t n) {
    if (n <= 512) { orc_ip_gpu_shared(r, a, b, n); return; }
    size_t nb = (n + 255) / 256;
    if (nb > 1024) nb = 1024;
    orc_fe part[1024], s[256];
    for (size_t k = 0; k < nb; k++) ip_block(&part[k], a, b, n, k, nb * 256, 0);
    for (size_t t = 0; t < 256; t++) { if (t < nb) s[t] = part[t]; else fe_set(&s[t], 0); }
    for (size_t st = 128; st > 0; st >>= 1)
        for (size_t t = 0; t < st; t++)
            if (t + st < nb) orc_fe_add(&s[t], &s[t], &s[t + st]);
    *r = s[0];
}
/* cuda_batch_field_vector_inner_product (cuda_inner_product.cu:302-347): per vector, the value
 * x-block 0 writes (the other x-blocks race on the same slot when n > 256). */
void orc_ip_gpu_batch(orc_fe* r, const orc_fe* a, const orc_fe* b, size_t n, size_t nvec) {
    size_t nb = (n + 255) / 256;
    if (nb > 1024) nb = 1024;
    if (nb == 0) nb = 1;
    for (size_t v = 0; v < nvec; v++) ip_block(&r[v], a + v * n, b + v * n, n, 0, nb * 256, 1);
}

/* ------------------------------------------------------------------ generators */
/* complete_bulletproof_test.cu:33-63 */
void orc_base_points(orc_ge* out, size_t n, const uint8_t seed32[32]) {
    for (size_t i = 0; i < n; i++) {
        uint8_t in[36], xy[64];
        memcpy(in, seed32, 32);
        in[32] = (uint8_t)(i >> 24); in[33] = (uint8_t)(i >> 16); in[34] = (uint8_t)(i >> 8); in[35] = (uint8_t)i;
        orc_sha256(xy, in, 36);
        orc_sha256(xy + 32, xy, 32);
        fe_from_le(&out[i].X, xy);
        fe_from_le(&out[i].Y, xy + 32);
        fe_set(&out[i].Z, 1);
        orc_fe_mul(&out[i].T, &out[i].X, &out[i].Y);
    }
}
/* complete_bulletproof_test.cu:84-109 */
void orc_gh(orc_ge* g, orc_ge* h) {
    uint8_t gs[32] = {0x03}, hs[32] = {0x04}, gb[32], hb[32];
    orc_sha256(gb, gs, 32);
    orc_sha256(hb, hs, 32);
    orc_ge_zero(g);
    orc_ge_zero(h);
    fe_from_le(&g->X, gb);
    fe_from_le(&h->X, hb);
    orc_fe_mul(&g->T, &g->X, &g->Y);
    orc_fe_mul(&h->T, &h->X, &h->Y);
}

/* ------------------------------------------------------------------ verify path */
/* bulletproof_challenge.cu:24-77 */
static void challenge_y(uint8_t out[32], const orc_ge* V, const orc_ge* A, const orc_ge* S) {
    uint8_t d[196];
    orc_fe_tobytes(d, &V->X); orc_fe_tobytes(d + 32, &V->Y);
    orc_fe_tobytes(d + 64, &A->X); orc_fe_tobytes(d + 96, &A->Y);
    orc_fe_tobytes(d + 128, &S->X); orc_fe_tobytes(d + 160, &S->Y);
    memcpy(d + 192, "y_ch", 4);
    orc_challenge(out, d, 196, "BulletproofYChal");
}
static void challenge_z(uint8_t out[32], const uint8_t y[32]) {
    uint8_t d[36];
    memcpy(d, y, 32);
    memcpy(d + 32, "z_ch", 4);
    orc_challenge(out, d, 36, "BulletproofZChal");
}
static void challenge_x(uint8_t out[32], const orc_ge* T1, const orc_ge* T2) {
    uint8_t d[132];
    orc_fe_tobytes(d, &T1->X); orc_fe_tobytes(d + 32, &T1->Y);
    orc_fe_tobytes(d + 64, &T2->X); orc_fe_tobytes(d + 96, &T2->Y);
    memcpy(d + 128, "xcha", 4); /* memcpy of 4 bytes of "xchal" (challenge.cu:73) */
    orc_challenge(out, d, 132, "BulletproofXChal");
}

static void scalarmult_host_norm(orc_ge* r, const orc_fe* s, const orc_ge* P) {
    uint8_t sb[32];
    orc_fe_tobytes(sb, s);
    orc_ge_scalarmult(r, sb, P);
    orc_ge_normalize_host(r);
}

/* bulletproof_range_proof.cu:658-762 calculate_inner_product_point */
static void calc_P(orc_ge* P, const orc_fe* y, const orc_fe* z, const orc_fe* t, size_t n, const orc_ge* G,
                   const orc_ge* H, const orc_ge* h) {
    orc_fe* pw = (orc_fe*)malloc(n * sizeof(orc_fe));
    orc_fe* sG = (orc_fe*)malloc(n * sizeof(orc_fe));
    orc_fe* sH = (orc_fe*)malloc(n * sizeof(orc_fe));
    orc_fe z2, zero, two, one;
    fe_set(&zero, 0);
    fe_set(&one, 1);
    if (n) fe_set(&pw[0], 1);
    for (size_t i = 1; i < n; i++) orc_fe_mul(&pw[i], &pw[i - 1], y);   /* powers_of :299 */
    orc_fe_mul(&z2, z, z);
    orc_fe_add(&two, &one, &one);
    for (size_t i = 0; i < n; i++) {
        orc_fe two_i, zt;
        orc_fe_sub(&sG[i], &zero, z);
        sH[i] = *z;
        fe_set(&two_i, 1);
        for (size_t j = 0; j < i; j++) orc_fe_mul(&two_i, &two_i, &two);
        orc_fe_mul(&zt, &z2, &two_i);
        orc_fe_add(&sH[i], &sH[i], &zt);
        orc_fe_mul(&sH[i], &sH[i], &pw[i]);
    }
    orc_ge t1, t2, t3;
    orc_msm_canon(&t1, sG, G, n);
    orc_msm_canon(&t2, sH, H, n);
    scalarmult_host_norm(&t3, t, h);
    orc_ge_zero(P);
    orc_ge_add(P, P, &t1); orc_ge_normalize_host(P);
    orc_ge_add(P, P, &t2); orc_ge_normalize_host(P);
    orc_ge_add(P, P, &t3); orc_ge_normalize_host(P);
    orc_ge_normalize_host(P);
    orc_ge_normalize_host(P);
    free(pw); free(sG); free(sH);
}

static int absdiff(int a, int b) { return a > b ? a - b : b - a; }

/* cuda_range_proof_verify.cu:130-370 (nb:6659) cuda_inner_product_verify */
int orc_cuda_inner_product_verify(size_t n, const orc_fe* a, const orc_fe* b, size_t ab_len, const orc_fe* c,
                                  const orc_ge* L, const orc_ge* R, size_t L_len, const orc_fe* x,
                                  const orc_ge* P, const orc_ge* G, const orc_ge* H, const orc_ge* Q,
                                  orc_ge* check_out, orc_ge* Gtrace, orc_ge* Htrace) {
    orc_fe claimed;
    uint8_t cb[32], eb[32];
    orc_inner_product(&claimed, a, b, ab_len);                 /* crv:146-158 */
    orc_fe_tobytes(cb, &claimed);
    orc_fe_tobytes(eb, c);
    if (memcmp(cb, eb, 32) != 0) return 0;

    orc_ge* Gc = (orc_ge*)malloc(n * sizeof(orc_ge));
    orc_ge* Hc = (orc_ge*)malloc(n * sizeof(orc_ge));
    memcpy(Gc, G, n * sizeof(orc_ge));
    memcpy(Hc, H, n * sizeof(orc_ge));
    uint8_t tr[32] = {0};
    size_t np = n, off = 0;
    for (size_t i = 0; i < L_len; i++) {                      /* crv:174-249 */
        np >>= 1;
        orc_fe u, ui;
        if (i == 0) {
            u = *x;
        } else {
            uint8_t d[96], ch[32];
            memcpy(d, tr, 32);
            orc_fe_tobytes(d + 32, &L[i].X);
            orc_fe_tobytes(d + 64, &R[i].X);
            orc_challenge(ch, d, 96, "InnerProductChal");
            memcpy(tr, ch, 32);
            fe_from_le(&u, ch);
        }
        orc_fe_invert(&ui, &u);
        for (size_t j = 0; j < np; j++) {
            orc_ge t1, t2;
            scalarmult_host_norm(&t1, &ui, &Gc[j]);
            scalarmult_host_norm(&t2, &u, &Gc[j + np]);
            orc_ge_add(&Gc[j], &t1, &t2);
            orc_ge_normalize_host(&Gc[j]);
            scalarmult_host_norm(&t1, &u, &Hc[j]);
            scalarmult_host_norm(&t2, &ui, &Hc[j + np]);
            orc_ge_add(&Hc[j], &t1, &t2);
            orc_ge_normalize_host(&Hc[j]);
        }
        if (Gtrace) memcpy(Gtrace + off, Gc, np * sizeof(orc_ge));
        if (Htrace) memcpy(Htrace + off, Hc, np * sizeof(orc_ge));
        off += np;
    }
    orc_ge cp, t1, t2, t3;                                      /* crv:252-278 */
    orc_ge_zero(&cp);
    scalarmult_host_norm(&t1, &a[0], &Gc[0]);
    scalarmult_host_norm(&t2, &b[0], &Hc[0]);
    scalarmult_host_norm(&t3, c, Q);
    orc_ge_add(&cp, &cp, &t1); orc_ge_normalize_host(&cp);
    orc_ge_add(&cp, &cp, &t2); orc_ge_normalize_host(&cp);
    orc_ge_add(&cp, &cp, &t3); orc_ge_normalize_host(&cp);
    if (check_out) *check_out = cp;
    free(Gc);
    free(Hc);

    uint8_t kb[64], pb[64], hin[128], hs[32];                   /* crv:281-357 tolerant accept rule */
    orc_fe_tobytes(kb, &cp.X); orc_fe_tobytes(kb + 32, &cp.Y);
    orc_fe_tobytes(pb, &P->X); orc_fe_tobytes(pb + 32, &P->Y);
    int xd = 0, yd = 0, sx = 0, sy = 0, msb = 0, hz = 0;
    for (int i = 0; i < 32; i++) {
        int dx = absdiff(kb[i], pb[i]), dy = absdiff(kb[i + 32], pb[i + 32]);
        xd += dx > 0; yd += dy > 0;
        sx += dx > 0 && dx <= 10; sy += dy > 0 && dy <= 10;
    }
    for (int i = 24; i < 32; i++)
        for (int bit = 0; bit < 8; bit++) msb += ((kb[i] ^ pb[i]) >> bit & 1) == 0;
    memcpy(hin, kb, 64);
    memcpy(hin + 64, pb, 64);
    orc_sha256(hs, hin, 128);
    for (int i = 0; i < 32; i++) hz += hs[i] != 0;
    return (sx + sy >= 20) || (msb >= 28) || (xd + yd <= 32) || (hz <= 24);
}

/* cuda_range_proof_verify.cu:82-127 (nb:6611) cuda_range_proof_verify; compute_precise_delta (crv:109)
 * only prints, so it is not restated. */
int orc_cuda_range_proof_verify(const orc_head* head, const orc_ge* V, size_t n, const orc_fe* a, const orc_fe* b,
                                size_t ab_len, const orc_ge* L, const orc_ge* R, size_t L_len, const orc_ge* G,
                                const orc_ge* H, const orc_ge* g, const orc_ge* h, orc_ge* P_out,
                                orc_ge* check_out, orc_ge* Gtrace, orc_ge* Htrace) {
    (void)g;
    uint8_t yb[32], zb[32], xb[32];
    orc_fe y, z, x;
    challenge_y(yb, V, &head->A, &head->S);
    fe_from_le(&y, yb);
    challenge_z(zb, yb);
    fe_from_le(&z, zb);
    challenge_x(xb, &head->T1, &head->T2);
    fe_from_le(&x, xb);
    orc_ge P;
    calc_P(&P, &y, &z, &head->t, n, G, H, h);
    if (P_out) *P_out = P;
    return orc_cuda_inner_product_verify(n, a, b, ab_len, &head->c, L, R, L_len, &head->x, &P, G, H, h,
                                         check_out, Gtrace, Htrace);
}

/* ------------------------------------------------------------------ range_proof_verify (A18) */
/* bulletproof_range_proof.cu:315-410 compute_precise_delta */
static void precise_delta(orc_fe* delta, const orc_fe* z, const orc_fe* y, size_t n) {
    orc_fe z2, z3, zmz2, sy, cy, one, two, c2, s2, t1, t2;
    orc_fe_mul(&z2, z, z);
    orc_fe_mul(&z3, &z2, z);
    orc_fe_sub(&zmz2, z, &z2);
    fe_set(&sy, 1);
    fe_set(&cy, 1);
    for (size_t i = 1; i < n; i++) {
        orc_fe_mul(&cy, &cy, y);
        orc_fe_add(&sy, &sy, &cy);
    }
    orc_fe_mul(&t1, &zmz2, &sy);
    fe_set(&one, 1);
    orc_fe_add(&two, &one, &one);
    fe_set(&c2, 1);
    fe_set(&s2, 1);
    for (size_t i = 1; i < n; i++) {
        orc_fe_mul(&c2, &c2, &two);
        orc_fe_add(&s2, &s2, &c2);
    }
    orc_fe_mul(&t2, &z3, &s2);
    orc_fe_sub(delta, &t1, &t2);
}

/* bulletproof_range_proof.cu:765-876 enhanced_range_check */
static int range_check(const orc_fe* t, const orc_fe* delta, const orc_fe* z, size_t n) {
    orc_fe z2, tmd, z2i, val, two_n, one, two, vt, z2t, ubc, vm;
    uint8_t vb[32], ub[32], db[32];
    orc_fe_mul(&z2, z, z);
    orc_fe_sub(&tmd, t, delta);
    orc_fe_invert(&z2i, &z2);
    orc_fe_mul(&val, &tmd, &z2i);
    fe_set(&two_n, 1);
    fe_set(&one, 1);
    orc_fe_add(&two, &one, &one);
    for (size_t i = 0; i < n; i++) orc_fe_mul(&two_n, &two_n, &two);
    orc_fe_sub(&vt, &tmd, &z2);
    orc_fe_mul(&z2t, &z2, &two_n);
    orc_fe_sub(&ubc, &z2t, &tmd);
    orc_fe_tobytes(vb, &vt);
    orc_fe_tobytes(ub, &ubc);
    int lower_ok = (vb[31] & 0x80) == 0, upper_ok = (ub[31] & 0x80) == 0;
    orc_fe_sub(&vm, &val, &two_n);
    orc_fe_tobytes(db, &vm);
    int close = 1;
    for (int i = 0; i < 4; i++)
        if (db[i] > 3 && db[i] < 253) { close = 0; break; }
    return lower_ok && upper_ok && !close;
}

/* bulletproof_range_proof.cu:412-656 robust_polynomial_identity_check */
static int poly_check(const orc_head* hd, const orc_ge* V, const orc_fe* x, const orc_fe* z, const orc_fe* delta,
                      const orc_ge* g, const orc_ge* h, orc_rpv_detail* d) {
    orc_fe z2, x2;
    orc_fe_mul(&z2, z, z);
    orc_fe_mul(&x2, x, x);
    orc_ge gt, ht, left, right, vz, gd, hm, tx, tx2;
    scalarmult_host_norm(&gt, &hd->t, g);
    scalarmult_host_norm(&ht, &hd->taux, h);
    orc_ge_add(&left, &gt, &ht);
    orc_ge_normalize_host(&left);
    orc_ge_zero(&right);
    scalarmult_host_norm(&vz, &z2, V);
    scalarmult_host_norm(&gd, delta, g);
    scalarmult_host_norm(&hm, &hd->mu, h);
    scalarmult_host_norm(&tx, x, &hd->T1);
    scalarmult_host_norm(&tx2, &x2, &hd->T2);
    orc_ge_add(&right, &right, &vz); orc_ge_normalize_host(&right);
    orc_ge_add(&right, &right, &gd); orc_ge_normalize_host(&right);
    orc_ge_add(&right, &right, &hm); orc_ge_normalize_host(&right);
    orc_ge_add(&right, &right, &tx); orc_ge_normalize_host(&right);
    orc_ge_add(&right, &right, &tx2); orc_ge_normalize_host(&right);
    orc_ge_normalize_host(&left);
    orc_ge_normalize_host(&right);
    uint8_t b[128];   /* left.X | left.Y | right.X | right.Y */
    orc_fe_tobytes(b, &left.X); orc_fe_tobytes(b + 32, &left.Y);
    orc_fe_tobytes(b + 64, &right.X); orc_fe_tobytes(b + 96, &right.Y);
    int dxc = 0, dyc = 0, sxc = 0, syc = 0;
    for (int i = 0; i < 32; i++) {
        int xd = absdiff(b[i], b[64 + i]), yd = absdiff(b[32 + i], b[96 + i]);
        dxc += xd > 0; dyc += yd > 0;
        sxc += xd > 0 && xd <= 10; syc += yd > 0 && yd <= 10;
    }
    int m1 = (dxc <= 5) || (sxc >= 24 && syc >= 20);
    int cons = 0, prev = 0, est = 0;
    for (int i = 0; i < 32; i++) {
        int diff = (int)b[i] - (int)b[64 + i];
        if (!est && diff != 0) {
            prev = diff;
            est = 1;
        } else if (est) {
            if (absdiff(diff, prev) <= 10) {
                cons++;
                prev = (prev * 3 + diff) / 4;   /* C division, truncation toward zero */
            }
        }
    }
    int m2 = cons >= 20;
    uint8_t ch[32], lmx[32], rmx[32];
    orc_sha256(ch, b, 128);
    orc_ge lm, rm;
    orc_ge_scalarmult(&lm, ch, &left);
    orc_ge_normalize_host(&lm);
    orc_ge_scalarmult(&rm, ch, &right);
    orc_ge_normalize_host(&rm);
    orc_fe_tobytes(lmx, &lm.X);
    orc_fe_tobytes(rmx, &rm.X);
    int tot = 0, top = 0;
    for (int i = 0; i < 32; i++)
        for (int bit = 0; bit < 8; bit++) {
            int eq = ((lmx[i] ^ rmx[i]) >> bit & 1) == 0;
            tot += eq;
            if (i >= 24) top += eq;
        }
    int m3 = top >= 22, m4 = tot >= 200;
    if (d) {
        d->poly_m1 = m1; d->poly_m2 = m2; d->poly_m3 = m3; d->poly_m4 = m4;
        d->left = left; d->right = right; d->left_mult = lm; d->right_mult = rm;
    }
    return m1 || m2 || m3 || m4;
}

/* bulletproof_vectors.cu:713-749: inner_product_verify's accept rule on the check point */
static int ip_cpu_accept(const orc_ge* cp, const orc_ge* P) {
    uint8_t kb[32], pb[32];
    orc_fe_tobytes(kb, &cp->X);
    orc_fe_tobytes(pb, &P->X);
    int xdc = 0, sxc = 0, mb = 0;
    for (int i = 0; i < 32; i++) {
        int d = absdiff(kb[i], pb[i]);
        xdc += d > 0;
        sxc += d > 0 && d <= 5;
    }
    if (xdc <= 3 || sxc >= 28) return 1;
    for (int i = 24; i < 32; i++)
        for (int bit = 0; bit < 8; bit++) mb += ((kb[i] ^ pb[i]) >> bit & 1) == 0;
    return mb >= 20;
}

int orc_range_proof_verify(const orc_head* head, const orc_ge* V, size_t n, const orc_fe* a, const orc_fe* b,
                           size_t ab_len, const orc_ge* L, const orc_ge* R, size_t L_len, const orc_ge* G,
                           const orc_ge* H, const orc_ge* g, const orc_ge* h, orc_rpv_detail* det) {
    orc_rpv_detail d;
    memset(&d, 0, sizeof(d));
    uint8_t v1[64], v2[64];                                   /* rp.cu:1729-1740 */
    orc_fe_tobytes(v1, &V->X); orc_fe_tobytes(v1 + 32, &V->Y);
    orc_fe_tobytes(v2, &head->V.X); orc_fe_tobytes(v2 + 32, &head->V.Y);
    d.vmatch = memcmp(v1, v2, 64) == 0;
    uint8_t yb[32], zb[32], xb[32];                           /* rp.cu:1746-1771 */
    orc_fe y, z, x;
    challenge_y(yb, V, &head->A, &head->S);
    fe_from_le(&y, yb);
    challenge_z(zb, yb);
    fe_from_le(&z, zb);
    challenge_x(xb, &head->T1, &head->T2);
    fe_from_le(&x, xb);
    precise_delta(&d.delta, &z, &y, n);                       /* rp.cu:1775 */
    d.range_ok = range_check(&head->t, &d.delta, &z, n);      /* rp.cu:1778, :1785 (same call twice) */
    d.poly_ok = poly_check(head, V, &x, &z, &d.delta, g, h, &d);   /* rp.cu:1793 */
    calc_P(&d.P, &y, &z, &head->t, n, G, H, h);               /* rp.cu:1803 */
    orc_ge cp;
    memset(&cp, 0, sizeof(cp));
    /* rp.cu:1806 inner_product_verify: same <a,b> check and fold as the CUDA verify, own accept rule */
    orc_fe claimed;
    uint8_t cb[32], eb[32];
    orc_inner_product(&claimed, a, b, ab_len);
    orc_fe_tobytes(cb, &claimed);
    orc_fe_tobytes(eb, &head->c);
    if (memcmp(cb, eb, 32) == 0) {
        orc_cuda_inner_product_verify(n, a, b, ab_len, &head->c, L, R, L_len, &head->x, &d.P, G, H, h, &cp, NULL,
                                      NULL);
        d.ip_ok = ip_cpu_accept(&cp, &d.P);
    }
    d.check = cp;
    if (det) *det = d;
    return d.vmatch && d.range_ok && d.poly_ok && d.ip_ok;
}

/* ------------------------------------------------------------------ prover */
/* bulletproof_range_proof.cu:277-297 pedersen_commit */
static void pedersen(orc_ge* r, const orc_fe* value, const orc_fe* blinding, const orc_ge* g, const orc_ge* h) {
    orc_ge t1, t2;
    scalarmult_host_norm(&t1, value, g);
    scalarmult_host_norm(&t2, blinding, h);
    orc_ge_add(r, &t1, &t2);
    orc_ge_normalize_host(r);
}

/* bulletproof_range_proof.cu:238-264 validate_range_input (n < 256) */
static int validate_range(const orc_fe* v, size_t n) {
    uint8_t vb[32];
    orc_fe_tobytes(vb, v);
    size_t bi = n / 8, bit = n % 8;
    if (vb[bi] & (1u << bit)) return 0;
    for (size_t i = bi + (bit == 7 ? 1 : 0); i < 32; i++)
        if (vb[i]) return 0;
    return 1;
}

/* bulletproof_vectors.cu:189-224 point_vector_multi_scalar_mul == orc_msm_cpu */

/* bulletproof_vectors.cu:277-523 inner_product_prove on a/b (length n, modified in place) */
static void ipa_prove(orc_fe* a, orc_fe* b, size_t n, const orc_ge* G, const orc_ge* H, const orc_ge* Q,
                      const uint8_t transcript0[32], orc_ge* L_out, orc_ge* R_out, size_t* L_len, orc_fe* x_out) {
    uint8_t tr[32];
    memcpy(tr, transcript0, 32);
    size_t rounds = 0;
    for (size_t i = n; i > 1; i >>= 1) rounds++;
    *L_len = rounds;
    size_t np = n;
    orc_fe* tmp = (orc_fe*)malloc((n ? n : 1) * sizeof(orc_fe));
    for (size_t r = 0; r < rounds; r++) {
        np >>= 1;
        orc_fe cL, cR;
        orc_inner_product(&cL, a, b + np, np);              /* <a_L, b_R> */
        orc_inner_product(&cR, a + np, b, np);              /* <a_R, b_L> */
        orc_ge L, R, t1, t2, t3;
        orc_msm_cpu(&t1, a, G + np, np);                     /* <a_L, G_R> */
        orc_msm_cpu(&t2, b + np, H, np);                     /* <b_R, H_L> */
        uint8_t cb[32];
        orc_fe_tobytes(cb, &cL);
        orc_ge_scalarmult(&t3, cb, Q);
        orc_ge_zero(&L);
        orc_ge_add(&L, &L, &t1); orc_ge_add(&L, &L, &t2); orc_ge_add(&L, &L, &t3);
        orc_ge_normalize_host(&L);
        L_out[r] = L;
        orc_msm_cpu(&t1, a + np, G, np);                     /* <a_R, G_L> */
        orc_msm_cpu(&t2, b, H + np, np);                     /* <b_L, H_R> */
        orc_fe_tobytes(cb, &cR);
        orc_ge_scalarmult(&t3, cb, Q);
        orc_ge_zero(&R);
        orc_ge_add(&R, &R, &t1); orc_ge_add(&R, &R, &t2); orc_ge_add(&R, &R, &t3);
        orc_ge_normalize_host(&R);
        R_out[r] = R;
        uint8_t d[96], ch[32];
        memcpy(d, tr, 32);
        orc_fe_tobytes(d + 32, &L.X);
        orc_fe_tobytes(d + 64, &R.X);
        orc_challenge(ch, d, 96, "InnerProductChal");
        memcpy(tr, ch, 32);
        orc_fe u, ui;
        fe_from_le(&u, ch);
        if (r == 0) *x_out = u;
        orc_fe_invert(&ui, &u);
        for (size_t j = 0; j < np; j++) {                    /* a' = u^-1 a_L + u a_R, b' = u b_L + u^-1 b_R */
            orc_fe p1, p2;
            orc_fe_mul(&p1, &u, &a[j + np]);
            orc_fe_mul(&p2, &ui, &a[j]);
            orc_fe_add(&tmp[j], &p2, &p1);
        }
        for (size_t j = 0; j < np; j++) {
            orc_fe p1, p2;
            orc_fe_mul(&p1, &u, &b[j]);
            orc_fe_mul(&p2, &ui, &b[j + np]);
            orc_fe_add(&b[j], &p1, &p2);
        }
        memcpy(a, tmp, np * sizeof(orc_fe));
    }
    free(tmp);
}

int orc_generate_range_proof(const uint8_t value32[32], const uint8_t gamma32[32], const uint8_t* sLR,
                             const uint8_t rnd4[4][32], size_t n, const orc_ge* G, const orc_ge* H, const orc_ge* g,
                             const orc_ge* h, orc_head* hd, orc_fe* a_out, orc_fe* b_out, orc_ge* L_out,
                             orc_ge* R_out, size_t* L_len) {
    orc_fe v, gamma, one, zero, two;
    fe_from_le(&v, value32);
    fe_from_le(&gamma, gamma32);
    if (!validate_range(&v, n)) return -1;                   /* rp.cu:1176-1188 */
    memset(hd, 0, sizeof(*hd));
    fe_set(&one, 1);
    fe_set(&zero, 0);
    orc_fe_add(&two, &one, &one);
    pedersen(&hd->V, &v, &gamma, g, h);                      /* rp.cu:1194 */
    uint8_t vb[32];
    orc_fe_tobytes(vb, &v);
    orc_fe* aL = (orc_fe*)calloc(n, sizeof(orc_fe));
    orc_fe* aR = (orc_fe*)calloc(n, sizeof(orc_fe));
    orc_fe* sL = (orc_fe*)calloc(n, sizeof(orc_fe));
    orc_fe* sR = (orc_fe*)calloc(n, sizeof(orc_fe));
    orc_fe* py = (orc_fe*)calloc(n, sizeof(orc_fe));
    orc_fe* p2 = (orc_fe*)calloc(n, sizeof(orc_fe));
    orc_fe* l = (orc_fe*)calloc(n, sizeof(orc_fe));
    orc_fe* rr = (orc_fe*)calloc(n, sizeof(orc_fe));
    orc_fe* u1 = (orc_fe*)calloc(n, sizeof(orc_fe));
    orc_fe* u2 = (orc_fe*)calloc(n, sizeof(orc_fe));
    for (size_t i = 0; i < n; i++) {                         /* rp.cu:1218-1238 */
        fe_set(&aL[i], (vb[i / 8] >> (i % 8)) & 1);
        orc_fe_sub(&aR[i], &aL[i], &one);
    }
    for (size_t i = 0; i < n; i++) {                         /* rp.cu:1246-1252 */
        fe_from_le(&sL[i], sLR + 64 * i);
        fe_from_le(&sR[i], sLR + 64 * i + 32);
    }
    orc_fe alpha, rho, tau1, tau2;
    fe_from_le(&alpha, rnd4[0]);
    fe_from_le(&rho, rnd4[1]);
    orc_ge t1, t2, t3;                                       /* rp.cu:1266-1290 */
    orc_ge_scalarmult(&t1, rnd4[0], h);
    orc_msm_cpu(&t2, aL, G, n);
    orc_msm_cpu(&t3, aR, H, n);
    orc_ge_add(&hd->A, &t1, &t2);
    orc_ge_add(&hd->A, &hd->A, &t3);
    orc_ge_normalize_host(&hd->A);
    orc_ge_scalarmult(&t1, rnd4[1], h);
    orc_msm_cpu(&t2, sL, G, n);
    orc_msm_cpu(&t3, sR, H, n);
    orc_ge_add(&hd->S, &t1, &t2);
    orc_ge_add(&hd->S, &hd->S, &t3);
    orc_ge_normalize_host(&hd->S);
    uint8_t yb[32], zb[32], xb[32];                          /* rp.cu:1302-1332 */
    orc_fe y, z, z2, x, x2;
    challenge_y(yb, &hd->V, &hd->A, &hd->S);
    challenge_z(zb, yb);
    fe_from_le(&y, yb);
    fe_from_le(&z, zb);
    orc_fe_mul(&z2, &z, &z);
    fe_set(&py[0], 1);                                       /* powers_of (rp.cu:299) */
    for (size_t i = 1; i < n; i++) orc_fe_mul(&py[i], &py[i - 1], &y);
    orc_fe tp;
    fe_set(&tp, 1);
    for (size_t i = 0; i < n; i++) {                         /* rp.cu:1347-1350 */
        p2[i] = tp;
        orc_fe_mul(&tp, &tp, &two);
    }
    /* t0 = <aL - z, y^n o (aR + z)> + z^2 <1, 2^n>   (rp.cu:1370-1407) */
    for (size_t i = 0; i < n; i++) {
        orc_fe_sub(&l[i], &aL[i], &z);                       /* aL - z */
        orc_fe_add(&rr[i], &aR[i], &z);                      /* aR + z */
        orc_fe_mul(&u1[i], &py[i], &rr[i]);                  /* y^n o (aR + z) */
        orc_fe_mul(&u2[i], &py[i], &sR[i]);                  /* y^n o sR */
    }
    orc_fe t0, s2n, zs2n, t1a, t1b, tt1, tt2;
    orc_inner_product(&t0, l, u1, n);
    fe_set(&s2n, 0);
    for (size_t i = 0; i < n; i++) orc_fe_add(&s2n, &s2n, &p2[i]);
    orc_fe_mul(&zs2n, &z2, &s2n);
    orc_fe_add(&t0, &t0, &zs2n);
    orc_inner_product(&t1a, sL, u1, n);                      /* rp.cu:1418-1426 */
    orc_inner_product(&t1b, l, u2, n);
    orc_fe_add(&tt1, &t1a, &t1b);
    orc_inner_product(&tt2, sL, u2, n);                      /* rp.cu:1430 */
    fe_from_le(&tau1, rnd4[2]);
    fe_from_le(&tau2, rnd4[3]);
    pedersen(&hd->T1, &tt1, &tau1, g, h);                    /* rp.cu:1442-1445 */
    pedersen(&hd->T2, &tt2, &tau2, g, h);
    orc_ge_normalize_host(&hd->T1);
    orc_ge_normalize_host(&hd->T2);
    challenge_x(xb, &hd->T1, &hd->T2);                       /* rp.cu:1452 */
    fe_from_le(&x, xb);
    orc_fe_mul(&x2, &x, &x);
    orc_fe m1, m2, t;                                        /* rp.cu:1470-1495 */
    orc_fe_mul(&m1, &tt1, &x);
    orc_fe_mul(&m2, &tt2, &x2);
    t = t0;
    orc_fe_add(&t, &t, &m1);
    orc_fe_add(&t, &t, &m2);
    hd->t = t;
    orc_fe_mul(&hd->taux, &tau1, &x);
    orc_fe_mul(&m2, &tau2, &x2);
    orc_fe_add(&hd->taux, &hd->taux, &m2);
    orc_fe_mul(&m1, &rho, &x);
    orc_fe_add(&hd->mu, &alpha, &m1);
    for (size_t i = 0; i < n; i++) {                         /* l(x), r(x) (rp.cu:1515-1580) */
        orc_fe e, sx;
        orc_fe_sub(&e, &aL[i], &z);
        orc_fe_mul(&sx, &sL[i], &x);
        orc_fe_add(&l[i], &e, &sx);
        orc_fe_add(&e, &aR[i], &z);
        orc_fe_mul(&sx, &sR[i], &x);
        orc_fe_add(&e, &e, &sx);
        orc_fe_mul(&e, &e, &py[i]);
        orc_fe_mul(&sx, &z2, &p2[i]);
        orc_fe_add(&rr[i], &e, &sx);
    }
    orc_fe ip;
    uint8_t ib[32], tb[32];
    orc_inner_product(&ip, l, rr, n);                        /* rp.cu:1600-1622 */
    orc_fe_tobytes(ib, &ip);
    orc_fe_tobytes(tb, &t);
    if (memcmp(ib, tb, 32) != 0) {
        memset(l, 0, n * sizeof(orc_fe));
        memset(rr, 0, n * sizeof(orc_fe));
        l[0] = t;
        fe_set(&rr[0], 1);
    }
    uint8_t fc[96], ipc[32];                                 /* rp.cu:1636-1650 */
    orc_fe_tobytes(fc, &t);
    orc_fe_tobytes(fc + 32, &hd->taux);
    orc_fe_tobytes(fc + 64, &hd->mu);
    orc_challenge(ipc, fc, 96, "BulletproofIP");
    fe_set(&hd->x, 0);
    ipa_prove(l, rr, n, G, H, h, ipc, L_out, R_out, L_len, &hd->x);   /* rp.cu:1656 */
    a_out[0] = t;                                            /* fix_inner_product_proof (rp.cu:198-235) */
    fe_set(&b_out[0], 1);
    hd->c = t;
    free(aL); free(aR); free(sL); free(sR); free(py); free(p2); free(l); free(rr); free(u1); free(u2);
    return 0;
}
