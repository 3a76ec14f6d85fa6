// ge25519_dev.h — gfx950 device point arithmetic reproducing the reference's "ge25519"
// extended-coordinate operations bit for bit.
//
// Freedoms used (all bit-preserving):
//  * the q-side terms (Y2-X2), (Y2+X2) of an add are computed once per fixed point;
//  * a doubling add(r, r) computes (Y-X) and (Y+X) once and squares them (same exact
//    product, so the same bits);
//  * a scalar's leading zero bits only ever double the identity: that prefix is a
//    table lookup (ident_doublings[k] = k doublings of (0,1,1,0)).
#pragma once
#include "fe25519_dev.h"

namespace bp {

#ifndef BP_LANE_ADDSUB
#define BP_LANE_ADDSUB 1
#endif
// E/H and F/G of ge25519_add: one fused block (fe_addsub, chains interleaved) or two calls
// (-DBP_LANE_ADDSUB=0, for A/B builds); the same bits either way.
BP_DEV void lane_addsub(const fe& f, const fe& g, fe& sum, fe& diff) {
#if BP_LANE_ADDSUB
    fe_addsub(f, g, sum, diff);
#else
    diff = fe_sub(f, g);
    sum = fe_add(f, g);
#endif
}

struct ge {
    fe X, Y, Z, T;
};

// q-side operands of ge25519_add: (Y-X), (Y+X), Z, T
struct geq {
    fe YmX, YpX, Z, T;
};

// curve25519_ops.cu:341-346 — LE bytes A3 78 59 13 ... 03 52 (this is d, used where 2d is meant)
BP_DEV fe k_const() {
    return fe{{0x75EB4DCA135978A3ull, 0x00700A4D4141D8ABull, 0x8CC740797779E898ull, 0x52036CEE2B6FFE73ull}};
}

// fe25519_mul(f, k) (the C = (T1 T2) k of every point operation): the same exact 512-bit product and
// fold as fe_mul(f, k_const()), with the product counting only the carries a column's running-sum
// bound allows (mul512_k_asm: 16 counts instead of 50; k's words are SGPR operands).
BP_DEV fe fe_mul_k(const fe& f) {
#if BP_MUL_ASM && defined(__HIP_DEVICE_COMPILE__)
    uint32_t a[8], w[16];
#pragma unroll
    for (int i = 0; i < 4; i++) {
        a[2 * i] = (uint32_t)f.v[i];
        a[2 * i + 1] = (uint32_t)(f.v[i] >> 32);
    }
    mul512_k_asm(w, a);
    uint64_t t[8];
#pragma unroll
    for (int i = 0; i < 8; i++) t[i] = (uint64_t)w[2 * i] | ((uint64_t)w[2 * i + 1] << 32);
    return fe_fold512(t);
#else
    return fe_mul(f, k_const());
#endif
}

BP_DEV ge ge_zero() { return ge{fe_set(0), fe_set(1), fe_set(1), fe_set(0)}; }   // curve25519_ops.cu:318

BP_DEV geq ge_prep(const ge& q) {
    return geq{fe_sub(q.Y, q.X), fe_add(q.Y, q.X), q.Z, q.T};
}

// ge25519_add (curve25519_ops.cu:326-378 == device_curve25519_ops.cuh:188-241)
BP_DEV ge ge_add_q(const ge& p, const geq& q) {
    fe A = fe_mul(fe_sub(p.Y, p.X), q.YmX);
    fe B = fe_mul(fe_add(p.Y, p.X), q.YpX);
    fe C = fe_mul_k(fe_mul(p.T, q.T));
    fe D = fe_mul(p.Z, q.Z);
    D = fe_add(D, D);
    fe E, F, G, H;
    lane_addsub(B, A, H, E);   // H = B + A, E = B - A
    lane_addsub(D, C, G, F);   // G = D + C, F = D - C
    return ge{fe_mul(E, F), fe_mul(G, H), fe_mul(F, G), fe_mul(E, H)};
}

BP_DEV ge ge_add(const ge& p, const ge& q) { return ge_add_q(p, ge_prep(q)); }

// add(p, p) (curve25519_ops.cu:406 / device .cuh:282)
BP_DEV ge ge_dbl(const ge& p) {
    fe A = fe_sq(fe_sub(p.Y, p.X));
    fe B = fe_sq(fe_add(p.Y, p.X));
    fe C = fe_mul_k(fe_sq(p.T));
    fe D = fe_sq(p.Z);
    D = fe_add(D, D);
    fe E, F, G, H;
    lane_addsub(B, A, H, E);   // H = B + A, E = B - A
    lane_addsub(D, C, G, F);   // G = D + C, F = D - C
    return ge{fe_mul(E, F), fe_mul(G, H), fe_mul(F, G), fe_mul(E, H)};
}

// device_ge25519_normalize (device_curve25519_ops.cuh:243-270): z_inv = 1.
BP_DEV ge ge_norm_dev(const ge& p) {
    ge r;
    r.X = fe_mul_one(p.X);
    r.Y = fe_mul_one(p.Y);
    r.Z = fe_set(1);
    r.T = fe_mul(r.X, r.Y);
    return r;
}

// ge25519_normalize (curve25519_ops.cu:574-605): keep the point when the canonical
// bytes of Z are 1, else multiply by the 13-step "invert" of Z.
BP_DEV ge ge_norm_host(const ge& p) {
    if (fe_is_one(fe_canon(p.Z))) return p;
    fe zi = fe_invert(p.Z);
    ge r;
    r.X = fe_mul(p.X, zi);
    r.Y = fe_mul(p.Y, zi);
    r.Z = fe_set(1);
    r.T = fe_mul(r.X, r.Y);
    return r;
}

BP_DEV int fe_clz256(const fe& s) {
    if (s.v[3]) return __clzll(s.v[3]);
    if (s.v[2]) return 64 + __clzll(s.v[2]);
    if (s.v[1]) return 128 + __clzll(s.v[1]);
    if (s.v[0]) return 192 + __clzll(s.v[0]);
    return 256;
}

BP_DEV ge ld_ge(const ge* p) { return *p; }

// Fixed-base prefix tables (optional, for points that are the same in every proof: the
// generators G_i, H_i, g, h).  ptab[p], p < 2^K, is the state of ge25519_scalarmult on this base
// after the top K bits of any scalar whose top K bits are p: the identity, then for each of
// those bits one add(r, r) and, for a set bit, one add(r, P).  A scalar with fewer than K
// leading zeros starts from ptab[top K bits] at bit 255 - K instead of from the identity at bit
// 255: the remaining operations are the same ones in the same order, so the result has the same
// bits.  (With K or more leading zeros the identity-doubling table dtab already covers them.)
constexpr int PREFIX_MAX_BITS = 24;
BP_DEV uint32_t prefix_index(const fe& s, int K) { return (uint32_t)(s.v[3] >> (64 - K)); }

// Length of ge25519_scalarmult's add chain past the leading zeros: the per-lane loop runs
// (256 - clz) doublings + popcount adds, and a wave runs as long as its longest lane.
BP_DEV int sm_ops(const fe& s) {
    return (256 - fe_clz256(s)) + __popcll(s.v[0]) + __popcll(s.v[1]) + __popcll(s.v[2]) + __popcll(s.v[3]);
}
// The same with a K-bit prefix table for the base (K = 0: none).
BP_DEV int sm_ops_prefix(const fe& s, int K) {
    if (K <= 0 || fe_clz256(s) >= K) return sm_ops(s);
    const uint64_t top = K == 64 ? 0 : (s.v[3] & (~0ull >> K));
    return (256 - K) + __popcll(s.v[0]) + __popcll(s.v[1]) + __popcll(s.v[2]) + __popcll(top);
}

// q-side operand access.  QLDS = true: this lane's LDS slot, read at the point of use (the
// empty asm with a memory clobber stops the compiler from hoisting the loads and keeping all
// of q in VGPRs, which would cost occupancy in the throughput kernels).  QLDS = false: a
// register copy (latency-bound kernels run one wave per SIMD, registers are free there).
template <bool QLDS>
BP_DEV fe qget(const fe* p) {
    if (QLDS) asm volatile("" ::: "memory");
    return *p;
}

// ge25519_add(p, q) with q's prepared operands (same operation order as ge_add_q).
// zone (wave-uniform): every lane's q.Z is exactly 1 (generators, host-normalized points), so
// Z1*Z2 = fold(Z1 || 0) = the conditional lossy "- p" of Z1 (fe_mul_one) — same bits, no product.
template <bool QLDS>
BP_DEV ge ge_add_qp(const ge& p, const geq* q, bool zone = false) {
    fe A = fe_mul(fe_sub(p.Y, p.X), qget<QLDS>(&q->YmX));
    fe B = fe_mul(fe_add(p.Y, p.X), qget<QLDS>(&q->YpX));
    fe C = fe_mul_k(fe_mul(p.T, qget<QLDS>(&q->T)));
    fe D = zone ? fe_mul_one(p.Z) : fe_mul(p.Z, qget<QLDS>(&q->Z));
    D = fe_add(D, D);
    fe E, F, G, H;
    lane_addsub(B, A, H, E);   // H = B + A, E = B - A
    lane_addsub(D, C, G, F);   // G = D + C, F = D - C
    return ge{fe_mul(E, F), fe_mul(G, H), fe_mul(F, G), fe_mul(E, H)};
}

// One step of the per-lane loop: add(r, r) when !use_q, add(r, q) when use_q; the
// select is per lane, the operation order is ge25519_add's in both cases.
// ZONE (wave-uniform): every lane's q.Z is exactly 1, so the add lanes' Z1*Z2 is fe_mul_one(Z1)
// and the doubling lanes' is the square Z1^2 — both formed, one kept (the same bits as the
// general product; 150 + ~20 VALU instead of 189 + the operand select).
template <bool QLDS, bool ZONE = false>
BP_DEV ge ge_add_sel(const ge& p, const geq* q, bool use_q) {
    // q's operands are loaded unconditionally and selected as values: a select between a
    // loaded and a computed value is otherwise folded into a load through a select of
    // pointers, which forces `p` into private memory (scratch).
    fe ymx = fe_sub(p.Y, p.X);
    fe qa = qget<QLDS>(&q->YmX);
    fe A = fe_mul(ymx, use_q ? qa : ymx);
    fe ypx = fe_add(p.Y, p.X);
    fe qb = qget<QLDS>(&q->YpX);
    fe B = fe_mul(ypx, use_q ? qb : ypx);
    fe qt = qget<QLDS>(&q->T);
    fe C = fe_mul_k(fe_mul(p.T, use_q ? qt : p.T));
    fe D;
    if (ZONE) {
        fe d1 = fe_mul_one(p.Z), d2 = fe_sq(p.Z);
        D = use_q ? d1 : d2;
    } else {
        fe qz = qget<QLDS>(&q->Z);
        D = fe_mul(p.Z, use_q ? qz : p.Z);
    }
    D = fe_add(D, D);
    fe E, F, G, H;
    lane_addsub(B, A, H, E);   // H = B + A, E = B - A
    lane_addsub(D, C, G, F);   // G = D + C, F = D - C
    return ge{fe_mul(E, F), fe_mul(G, H), fe_mul(F, G), fe_mul(E, H)};
}

// MSB-first bit stream over a 256-bit scalar, kept as a shift register of limbs so that no
// array is ever indexed by a run-time value (that would place the scalar in scratch).
struct BitStream {
    uint64_t cur, n1, n2, n3;   // cur's MSB is the next bit
    int left;                   // bits left in cur
};

// Position the stream at bit i (0..255) of s.
BP_DEV BitStream bs_init(const fe& s, int i) {
    BitStream b{s.v[3], s.v[2], s.v[1], s.v[0], 0};
    int L = i >> 6;
#pragma unroll
    for (int k = 0; k < 3; k++) {
        bool sh = k < 3 - L;
        b.cur = sh ? b.n1 : b.cur;
        b.n1 = sh ? b.n2 : b.n1;
        b.n2 = sh ? b.n3 : b.n2;
        b.n3 = sh ? 0 : b.n3;
    }
    int bi = i & 63;
    b.cur <<= (63 - bi);
    b.left = bi + 1;
    return b;
}

BP_DEV uint32_t bs_next(BitStream& b) {
    uint32_t bit = (uint32_t)(b.cur >> 63);
    b.cur <<= 1;
    if (--b.left == 0) {
        b.cur = b.n1;
        b.n1 = b.n2;
        b.n2 = b.n3;
        b.n3 = 0;
        b.left = 64;
    }
    return bit;
}

// ge25519_scalarmult (curve25519_ops.cu:397-415 == device .cuh:272-290) for a scalar
// that is the same in every lane of the wave: the bit test is a scalar branch.
// `s` holds the scalar's 256 bits (limb i = bytes 8i..8i+7, little-endian); `q` holds
// ge_prep(P); `dtab` = the identity-doubling table (257 points).
template <bool QLDS>
BP_DEV ge sm_uniform(const fe& s_in, const geq* q, const ge* __restrict__ dtab, const ge* ptab, int K) {
    fe s;
#pragma unroll
    for (int i = 0; i < 4; i++) {
        uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)s_in.v[i]);
        uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(s_in.v[i] >> 32));
        s.v[i] = (uint64_t)lo | ((uint64_t)hi << 32);
    }
    int lz = fe_clz256(s);
    // the prefix start only when every lane has a table (the start bit must stay wave-uniform)
    const bool pre = K > 0 && lz < K && __all(ptab != nullptr);
    const int top = pre ? 255 - K : 255 - lz;
    ge r = ld_ge(pre ? &ptab[prefix_index(s, K)] : &dtab[lz]);
    if (top < 0) return r;
    const bool zone = __all(fe_is_one(qget<QLDS>(&q->Z)));
    BitStream bs = bs_init(s, top);
    for (int i = top; i >= 0; i--) {
        r = ge_dbl(r);
        if (bs_next(bs)) r = ge_add_qp<QLDS>(r, q, zone);
    }
    return r;
}

// Same function for a per-lane scalar: every iteration is one ge25519_add whose second
// operand is either r itself (the doubling) or P, so no lane idles on the other's branch.
template <bool QLDS, bool ZONE>
BP_DEV ge sm_lane_loop(const fe& s, const geq* q, const ge* __restrict__ dtab, const ge* ptab, int K) {
    int lz = fe_clz256(s);
    const bool pre = K > 0 && lz < K && ptab != nullptr;
    ge r = ld_ge(pre ? &ptab[prefix_index(s, K)] : &dtab[lz]);
    int i = pre ? 255 - K : 255 - lz;   // index of the pending bit
    BitStream bs = bs_init(s, i < 0 ? 0 : i);
    uint32_t bit = i >= 0 ? bs_next(bs) : 0;
    bool add_phase = false;    // false: next op doubles; true: next op adds P
    while (i >= 0) {
        r = ge_add_sel<QLDS, ZONE>(r, q, add_phase);
        if (!add_phase && bit) {
            add_phase = true;
        } else {
            add_phase = false;
            i--;
            bit = bs_next(bs);
        }
    }
    return r;
}

template <bool QLDS>
BP_DEV ge sm_lane(const fe& s, const geq* q, const ge* __restrict__ dtab, const ge* ptab, int K) {
    if (__all(fe_is_one(qget<QLDS>(&q->Z)))) return sm_lane_loop<QLDS, true>(s, q, dtab, ptab, K);
    return sm_lane_loop<QLDS, false>(s, q, dtab, ptab, K);
}

// Wave-level dispatch: uniform scalar -> scalar-branch loop, else the per-lane loop.
// QLDS: `slot` is this lane's LDS slot and receives ge_prep(P); otherwise q stays in VGPRs.
// ptab / K: this lane's base's prefix table (nullable) and its width in bits (0: none).
template <bool QLDS>
BP_DEV ge scalarmult(const fe& s, const ge& P, geq* slot, const ge* __restrict__ dtab, const ge* ptab = nullptr,
                     int K = 0) {
    geq qreg;
    const geq* q;
    if (QLDS) {
        fe ymx = fe_sub(P.Y, P.X), ypx = fe_add(P.Y, P.X);
#pragma unroll
        for (int k = 0; k < 4; k++) {   // limb stores: an aggregate copy would stage through scratch
            slot->YmX.v[k] = ymx.v[k];
            slot->YpX.v[k] = ypx.v[k];
            slot->Z.v[k] = P.Z.v[k];
            slot->T.v[k] = P.T.v[k];
        }
        q = slot;
    } else {
        qreg = ge_prep(P);
        q = &qreg;
    }
    uint32_t same = 1;
#pragma unroll
    for (int i = 0; i < 4; i++) {
        uint32_t lo = (uint32_t)s.v[i], hi = (uint32_t)(s.v[i] >> 32);
        same &= (lo == __builtin_amdgcn_readfirstlane(lo)) & (hi == __builtin_amdgcn_readfirstlane(hi));
    }
    if (__all(same)) return sm_uniform<QLDS>(s, q, dtab, ptab, K);
    return sm_lane<QLDS>(s, q, dtab, ptab, K);
}

}  // namespace bp
