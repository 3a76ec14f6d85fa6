// fe25519_dev.h — gfx950 device arithmetic for the reference's "fe25519" field elements.
//
// The reference arithmetic is NOT GF(2^255-19): every routine here
// reproduces the exact bits of curve25519_ops.cu / device_curve25519_ops.cuh,
// including the lossy borrow chains and the truncated 19x fold. Only the ways the
// same bits are computed are free: the 512-bit product is formed by 32x32->64
// multiply-accumulates (product scanning), the "- p" fix-up is a closed form of the
// reference's borrow loop, and the tobytes/normalize early-outs are branch-free.
//
// Layout: 4 little-endian u64 limbs (curve25519_ops.h:15-17) kept in VGPR pairs.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#ifndef BP_MUL_ASM
#define BP_MUL_ASM 1
#endif
#include "mul512_asm.h"
#ifndef BP_FIELD_ASM
#define BP_FIELD_ASM 1
#endif
#include "field_asm.h"

namespace bp {

struct fe {
    uint64_t v[4];
};

#define BP_DEV __host__ __device__ __forceinline__

constexpr uint64_t P0 = 0xFFFFFFFFFFFFFFEDull;   // curve25519_ops.cu:7-8
constexpr uint64_t P3 = 0x7FFFFFFFFFFFFFFFull;
constexpr uint64_t M64 = 0xFFFFFFFFFFFFFFFFull;

BP_DEV fe fe_set(uint64_t x) { return fe{{x, 0, 0, 0}}; }

// t >= p, lexicographic from limb 3 (curve25519_ops.cu:54-59). p1 = p2 = 2^64-1.
BP_DEV bool fe_ge_p(const fe& t) {
    bool top = (t.v[3] >> 63) != 0;
    bool eq = (t.v[3] == P3) & (t.v[2] == M64) & (t.v[1] == M64) & (t.v[0] >= P0);
    return top | eq;
}

// The reference's "- p" loop (curve25519_ops.cu:62-66 / :137-141 / :232-237):
//   diff = h_i - p_i - br;  br = h_i < lo64(p_i + br)
// For p1 = p2 = 2^64-1 the sum p_i + br wraps to 0 when br = 1, dropping the borrow.
// Closed form of the same four steps:
BP_DEV fe fe_lossy_sub_p(const fe& t) {
    fe d;
    uint64_t br1 = t.v[0] < P0;
    d.v[0] = t.v[0] + 19;                         // t0 - (2^64 - 19)
    d.v[1] = t.v[1] + 1 - br1;                    // t1 - (2^64 - 1) - br1
    uint64_t br2 = (br1 == 0) & (t.v[1] != M64);
    d.v[2] = t.v[2] + 1 - br2;
    uint64_t br3 = (br2 == 0) & (t.v[2] != M64);
    d.v[3] = t.v[3] - P3 - br3;
    return d;
}

// m ? lossy_sub_p(t) : t, folded into the additions: with br1 = t0 < p0,
// br2 = !br1 & t1 != 2^64-1, br3 = !br2 & t2 != 2^64-1 (the closed form above),
//   out = t + m*(19, !br1, !br2, 2^63 + !br3)   (mod 2^64 per limb, no carries between limbs).
BP_DEV fe fe_cond_sub_p(const fe& t, bool m) {
    bool br1 = t.v[0] < P0;
    bool br2 = !br1 & (t.v[1] != M64);
    bool br3 = !br2 & (t.v[2] != M64);
    fe o;
    o.v[0] = t.v[0] + (m ? 19ull : 0ull);
    o.v[1] = t.v[1] + (uint64_t)(m & !br1);
    o.v[2] = t.v[2] + (uint64_t)(m & !br2);
    o.v[3] = t.v[3] + (m ? (0x8000000000000000ull + (uint64_t)!br3) : 0ull);
    return o;
}

// The fix-up shared by add and the product fold: (carry || t >= p) ? lossy_sub_p(t) : t,
// with the compare masks of t >= p (curve25519_ops.cu:54-59) and of the borrow chain shared.
BP_DEV fe fe_fix(const fe& t, bool carry) {
    bool lt0 = t.v[0] < P0;              // br1
    bool f1 = t.v[1] == M64, f2 = t.v[2] == M64;
    bool top = (int64_t)t.v[3] < 0;
    bool e3 = t.v[3] == P3;
    bool m = carry | top | (e3 & f2 & f1 & !lt0);
    bool br2 = !lt0 & !f1;
    bool br3 = !br2 & !f2;
    fe o;
    o.v[0] = t.v[0] + (m ? 19ull : 0ull);
    o.v[1] = t.v[1] + (uint64_t)(m & !lt0);
    o.v[2] = t.v[2] + (uint64_t)(m & !br2);
    o.v[3] = t.v[3] + (m ? (0x8000000000000000ull + (uint64_t)!br3) : 0ull);
    return o;
}

// lo64(19 x) as two shift-adds (x + 16x, then + 2x).
BP_DEV uint64_t mul19(uint64_t x) {
#ifdef __HIP_DEVICE_COMPILE__
    uint64_t y, z;
    asm("v_lshl_add_u64 %0, %1, 4, %1" : "=v"(y) : "v"(x));
    asm("v_lshl_add_u64 %0, %1, 1, %2" : "=v"(z) : "v"(x), "v"(y));
    return z;
#else
    return x * 19ull;
#endif
}

// host fe25519_tobytes (curve25519_ops.cu:220-251) minus the byte store: canonicalising limbs.
BP_DEV fe fe_canon(const fe& t) {
#if BP_FIELD_ASM && defined(__HIP_DEVICE_COMPILE__)   // generated gfx950 form (field_asm.h), same bits
    uint32_t a[8], o[8];
#pragma unroll
    for (int i = 0; i < 4; i++) {
        a[2 * i] = (uint32_t)t.v[i];
        a[2 * i + 1] = (uint32_t)(t.v[i] >> 32);
    }
    fe_canon_asm(o, a);
    return fe{{(uint64_t)o[0] | ((uint64_t)o[1] << 32), (uint64_t)o[2] | ((uint64_t)o[3] << 32),
               (uint64_t)o[4] | ((uint64_t)o[5] << 32), (uint64_t)o[6] | ((uint64_t)o[7] << 32)}};
#else
    return fe_cond_sub_p(t, fe_ge_p(t));
#endif
}

BP_DEV uint32_t lo32(uint64_t x) { return (uint32_t)x; }
BP_DEV uint32_t hi32(uint64_t x) { return (uint32_t)(x >> 32); }
BP_DEV uint64_t cat64(uint32_t lo, uint32_t hi) { return (uint64_t)lo | ((uint64_t)hi << 32); }

// fe25519_add (curve25519_ops.cu:41-68): exact 257-bit sum (one 32-bit carry chain), then
// one lossy "- p" when the sum carried out or is >= p.
// LAT 1: the latency form of the generated block (field_asm.h fe_add_asm_lat, the 16-lane row step);
// LAT 2: its fast statement alone, the rare-edge test deferred into *acc (fe_add_asm_lat_acc).
template <int LAT = 0>
BP_DEV fe fe_add(const fe& f, const fe& g, uint32_t* acc = nullptr) {
#if BP_FIELD_ASM && defined(__HIP_DEVICE_COMPILE__)   // generated gfx950 form (field_asm.h), same bits
    uint32_t a[8], b[8], o[8];
#pragma unroll
    for (int i = 0; i < 4; i++) {
        a[2 * i] = lo32(f.v[i]); a[2 * i + 1] = hi32(f.v[i]);
        b[2 * i] = lo32(g.v[i]); b[2 * i + 1] = hi32(g.v[i]);
    }
    if constexpr (LAT == 2) fe_add_asm_lat_acc(o, a, b, *acc); else if constexpr (LAT == 1) fe_add_asm_lat(o, a, b); else fe_add_asm(o, a, b);
    return fe{{cat64(o[0], o[1]), cat64(o[2], o[3]), cat64(o[4], o[5]), cat64(o[6], o[7])}};
#else
    fe h;
    unsigned c = 0;
#pragma unroll
    for (int i = 0; i < 4; i++) {
        uint32_t l = __builtin_addc(lo32(f.v[i]), lo32(g.v[i]), c, &c);
        uint32_t u = __builtin_addc(hi32(f.v[i]), hi32(g.v[i]), c, &c);
        h.v[i] = cat64(l, u);
    }
    return fe_fix(h, c != 0);
#endif
}

// fe25519_sub (curve25519_ops.cu:71-90): t_i = f_i - g_i - br;  br = f_i < lo64(g_i + br).
// The lossy borrow equals the true borrow except when g_i = 2^64-1 and br = 1 (g_i + br wraps
// to 0 and the borrow is dropped).  Then, on a final borrow, the literal "+ p" pass:
//   a0 = t0 + p0, cy = a0 < p0 (= t0 >= 19);  a_i = t_i + lo64(p_i + cy), cy = a_i < p_i
// i.e. a_i = cy ? t_i : t_i - 1 and cy = a_i != 2^64-1 for i = 1, 2;  a3 = t3 + p3 + cy.
BP_DEV fe fe_sub(const fe& f, const fe& g) {
#if BP_FIELD_ASM && defined(__HIP_DEVICE_COMPILE__)   // generated gfx950 form (field_asm.h), same bits
    uint32_t a[8], b[8], o[8];
#pragma unroll
    for (int i = 0; i < 4; i++) {
        a[2 * i] = lo32(f.v[i]); a[2 * i + 1] = hi32(f.v[i]);
        b[2 * i] = lo32(g.v[i]); b[2 * i + 1] = hi32(g.v[i]);
    }
    fe_sub_asm(o, a, b);
    return fe{{cat64(o[0], o[1]), cat64(o[2], o[3]), cat64(o[4], o[5]), cat64(o[6], o[7])}};
#else
    fe t;
    unsigned br = 0;
#pragma unroll
    for (int i = 0; i < 4; i++) {
        unsigned b1, b2;
        uint32_t l = __builtin_subc(lo32(f.v[i]), lo32(g.v[i]), br, &b1);
        uint32_t u = __builtin_subc(hi32(f.v[i]), hi32(g.v[i]), b1, &b2);
        t.v[i] = cat64(l, u);
        br = b2 & !((g.v[i] == M64) & (br != 0));
    }
    const bool m = br != 0;
    fe o;
    o.v[0] = t.v[0] - (m ? 19ull : 0ull);
    bool cy0 = t.v[0] >= 19;
    o.v[1] = t.v[1] - (uint64_t)(m & !cy0);
    bool cy1 = o.v[1] != M64;
    o.v[2] = t.v[2] - (uint64_t)(m & !cy1);
    bool cy2 = o.v[2] != M64;
    o.v[3] = t.v[3] + (m ? (cy2 ? 0x8000000000000000ull : P3) : 0ull);
    return o;
#endif
}

// fe_add(f, g) and fe_sub(f, g) together (the generated block interleaves the two carry chains:
// fewer wait states in the latency-bound lane-quad chains); the same bits as the two calls.
template <int LAT = 0>
BP_DEV void fe_addsub(const fe& f, const fe& g, fe& sum, fe& diff, uint32_t* acc = nullptr) {
#if BP_FIELD_ASM && defined(__HIP_DEVICE_COMPILE__)
    uint32_t a[8], b[8], os[8], od[8];
#pragma unroll
    for (int i = 0; i < 4; i++) {
        a[2 * i] = lo32(f.v[i]); a[2 * i + 1] = hi32(f.v[i]);
        b[2 * i] = lo32(g.v[i]); b[2 * i + 1] = hi32(g.v[i]);
    }
    if constexpr (LAT == 2) fe_addsub_asm_lat_acc(os, od, a, b, *acc);
    else if constexpr (LAT == 1) fe_addsub_asm_lat(os, od, a, b);
    else fe_addsub_asm(os, od, a, b);
    sum = fe{{cat64(os[0], os[1]), cat64(os[2], os[3]), cat64(os[4], os[5]), cat64(os[6], os[7])}};
    diff = fe{{cat64(od[0], od[1]), cat64(od[2], od[3]), cat64(od[4], od[5]), cat64(od[6], od[7])}};
#else
    sum = fe_add(f, g);
    diff = fe_sub(f, g);
#endif
}

// Fold of the exact 512-bit product (curve25519_ops.cu:114-145):
//   c = lo64(t4*19); t0 += c; cy = t0 < c;
//   c = lo64(t_{i+4}*19 + cy); t_i += c; cy = t_i < c   (i = 1..3)
//   if (cy || t >= p) lossy "- p"
// Computed as one carry chain t_i + x_i + cy (x_i = lo64(19 t_{i+4})): the same sum; the
// carry differs only when x_i = 2^64-1 and cy = 1 (c wraps to 0, the reference carries 0).
template <int LAT = 0>
BP_DEV fe fe_fold512(const uint64_t t[8], uint32_t* acc = nullptr) {
#if BP_FIELD_ASM && defined(__HIP_DEVICE_COMPILE__)   // generated gfx950 form (field_asm.h), same bits
    uint32_t a[8], xh[8], o[8];
#pragma unroll
    for (int i = 0; i < 4; i++) {
        uint64_t x = mul19(t[i + 4]);
        a[2 * i] = lo32(t[i]); a[2 * i + 1] = hi32(t[i]);
        xh[2 * i] = lo32(x); xh[2 * i + 1] = hi32(x);
    }
    if constexpr (LAT == 2) fe_fold_asm_lat_acc(o, a, xh, *acc); else if constexpr (LAT == 1) fe_fold_asm_lat(o, a, xh); else fe_fold_asm(o, a, xh);
    return fe{{cat64(o[0], o[1]), cat64(o[2], o[3]), cat64(o[4], o[5]), cat64(o[6], o[7])}};
#else
    fe h;
    unsigned cy = 0;
#pragma unroll
    for (int i = 0; i < 4; i++) {
        uint64_t x = mul19(t[i + 4]);
        unsigned k, c;
        uint32_t l = __builtin_addc(lo32(t[i]), lo32(x), cy, &k);
        uint32_t u = __builtin_addc(hi32(t[i]), hi32(x), k, &c);
        h.v[i] = cat64(l, u);
        cy = c & !((x == M64) & (cy != 0));
    }
    return fe_fix(h, cy != 0);
#endif
}

// Exact 256x256 -> 512-bit product, product scanning over 32-bit words with a
// 96-bit column accumulator.  BP_MUL_ASM selects the generated gfx950 column kernels
// (mul512_asm.h: v_mad_u64_u32 carry-out + v_addc_co_u32, 2 VALU per 32x32 product);
// the plain-C form below is the reference formulation of the same product.
BP_DEV void mul512(uint64_t t[8], const fe& f, const fe& g) {
    uint32_t a[8], b[8], w[16];
#pragma unroll
    for (int i = 0; i < 4; i++) {
        a[2 * i] = (uint32_t)f.v[i];
        a[2 * i + 1] = (uint32_t)(f.v[i] >> 32);
        b[2 * i] = (uint32_t)g.v[i];
        b[2 * i + 1] = (uint32_t)(g.v[i] >> 32);
    }
#if BP_MUL_ASM && defined(__HIP_DEVICE_COMPILE__)   // host pass: the C form (host-side checks)
    // bounded form (the first carry of every column uncounted, mul512_asm.h) unless a lane's gating
    // words a[0], b[7] exceed MUL_BOUNDED_WORD (a wave-uniform test; ~2^-27 per lane): then the
    // counting form recomputes the product (out of line).  (A form that also left the second carry
    // of columns 7..13 uncounted, gated on top words <= 0x7FFFFFEF, ran at 123 K vs 202 K verifies/s:
    // this arithmetic's values are not reduced below 2^255, so that gate failed in most waves,
    // profiles/ab/r05d_bounded2.json.)
    mul512_bounded_asm(w, a, b);
    if (__builtin_expect(__any(max(a[0], b[7]) > MUL_BOUNDED_WORD), 0)) mul512_asm(w, a, b);
#else
    uint64_t acc = 0;
    uint32_t c2 = 0;
#pragma unroll
    for (int k = 0; k < 15; k++) {
#pragma unroll
        for (int i = 0; i < 8; i++) {
            int j = k - i;
            if (j < 0 || j > 7) continue;
            uint64_t p = (uint64_t)a[i] * b[j];
            acc += p;
            c2 += acc < p;
        }
        w[k] = (uint32_t)acc;
        acc = (acc >> 32) | ((uint64_t)c2 << 32);
        c2 = 0;
    }
    w[15] = (uint32_t)acc;
#endif
#pragma unroll
    for (int i = 0; i < 8; i++) t[i] = (uint64_t)w[2 * i] | ((uint64_t)w[2 * i + 1] << 32);
}

// fe25519_mul (curve25519_ops.cu:93-146 == device_curve25519_ops.cuh:117-171)
BP_DEV fe fe_mul(const fe& f, const fe& g) {
    uint64_t t[8];
    mul512(t, f, g);
    return fe_fold512(t);
}

// Exact 512-bit square: 2 * (off-diagonal products, 28 of them) + the 8 diagonal squares —
// the same 512 bits as mul512(t, f, f) with 36 instead of 64 32x32 products.
BP_DEV void sqr512(uint64_t t[8], const fe& f) {
    uint32_t a[8], o[16], w[16];
#pragma unroll
    for (int i = 0; i < 4; i++) {
        a[2 * i] = (uint32_t)f.v[i];
        a[2 * i + 1] = (uint32_t)(f.v[i] >> 32);
    }
#if BP_MUL_ASM && defined(__HIP_DEVICE_COMPILE__)
    sqr512_offdiag_bounded_asm(o, a);
    if (__builtin_expect(__any(max(a[0], a[7]) > MUL_BOUNDED_WORD), 0)) sqr512_offdiag_asm(o, a);
#else
    uint64_t acc = 0;
    uint32_t c2 = 0;
    o[0] = 0;
#pragma unroll
    for (int k = 1; k < 14; k++) {
#pragma unroll
        for (int i = 0; i < 8; i++) {
            int j = k - i;
            if (j <= i || j > 7) continue;
            uint64_t p = (uint64_t)a[i] * a[j];
            acc += p;
            c2 += acc < p;
        }
        o[k] = (uint32_t)acc;
        acc = (acc >> 32) | ((uint64_t)c2 << 32);
        c2 = 0;
    }
    o[14] = (uint32_t)acc;
    o[15] = (uint32_t)(acc >> 32);
#endif
    // w = 2 o + sum a_i^2 2^(64 i): one carry chain over the doubled words (funnel shifts)
    unsigned c = 0;
    uint64_t d0 = (uint64_t)a[0] * a[0];
    w[0] = (uint32_t)d0;
    w[1] = __builtin_addc(o[1] << 1, (uint32_t)(d0 >> 32), 0u, &c);
#pragma unroll
    for (int i = 1; i < 8; i++) {
        uint64_t di = (uint64_t)a[i] * a[i];
        uint32_t lo = (o[2 * i] << 1) | (o[2 * i - 1] >> 31);
        uint32_t hi = (o[2 * i + 1] << 1) | (o[2 * i] >> 31);
        w[2 * i] = __builtin_addc(lo, (uint32_t)di, c, &c);
        w[2 * i + 1] = __builtin_addc(hi, (uint32_t)(di >> 32), c, &c);
    }
#pragma unroll
    for (int i = 0; i < 8; i++) t[i] = (uint64_t)w[2 * i] | ((uint64_t)w[2 * i + 1] << 32);
}

// fe25519_sq (curve25519_ops.cu:149) == mul(f, f): the same exact product, then the same fold.
BP_DEV fe fe_sq(const fe& f) {
    uint64_t t[8];
    sqr512(t, f);
    return fe_fold512(t);
}

// mul by 1 (device_curve25519_ops.cuh:260 with z_inv = 1): product has zero upper half,
// the fold adds nothing, so it is the conditional lossy "- p".
BP_DEV fe fe_mul_one(const fe& f) { return fe_canon(f); }

// fe25519_invert (curve25519_ops.cu:157-207): the fixed 13-multiplication chain.
// t2 = sq(f) at :198 equals t0's first value (:163), so it is reused (12 products).
BP_DEV fe fe_invert(const fe& f) {
    fe f2 = fe_sq(f);              // :163 t0 = f^2
    fe t1 = fe_sq(f2);             // :166
    t1 = fe_sq(t1);                // :169
    t1 = fe_mul(t1, f);            // :172
    fe t0 = fe_mul(t1, f2);        // :175
    t1 = fe_sq(t0);                // :178
    t1 = fe_sq(t1);                // :186
    t1 = fe_sq(t1);                // :189
    t1 = fe_sq(t1);                // :192
    t1 = fe_mul(t1, t1);           // :195
    fe t2 = fe_mul(f2, f);         // :198-199 (sq(f) reused)
    return fe_mul(t1, t2);         // :200
}

BP_DEV bool fe_is_one(const fe& f) {
    return (f.v[0] == 1) & (f.v[1] == 0) & (f.v[2] == 0) & (f.v[3] == 0);
}

BP_DEV bool fe_eq(const fe& a, const fe& b) {
    return (a.v[0] == b.v[0]) & (a.v[1] == b.v[1]) & (a.v[2] == b.v[2]) & (a.v[3] == b.v[3]);
}

// The reference's "square" GPU kernel (cuda_field_ops.cu:147-216): carries between
// limbs are dropped and 2*a_i*a_j is taken mod 2^128. It is not fe25519_sq;
// reproduced for the cuda_batch_field_square entry point.
BP_DEV fe fe_square_kernel_quirk(const fe& f) {
    uint64_t t[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
    for (int i = 0; i < 4; i++) {
        unsigned __int128 d = (unsigned __int128)f.v[i] * f.v[i];
        t[2 * i] += (uint64_t)d;
        if (2 * i + 1 < 8) t[2 * i + 1] += (uint64_t)(d >> 64);
#pragma unroll
        for (int j = i + 1; j < 4; j++) {
            unsigned __int128 m = ((unsigned __int128)f.v[i] * f.v[j]) << 1;
            t[i + j] += (uint64_t)m;
            if (i + j + 1 < 8) t[i + j + 1] += (uint64_t)(m >> 64);
        }
    }
    return fe_fold512(t);
}

BP_DEV uint32_t fe_byte(const fe& f, int i) { return (uint32_t)(f.v[i >> 3] >> (8 * (i & 7))) & 0xff; }

BP_DEV uint32_t fe_bit(const fe& s, int i) { return (uint32_t)(s.v[i >> 6] >> (i & 63)) & 1u; }

}  // namespace bp
