// ge25519_quad.h — point operations spread over a lane QUAD, for latency-bound chains (the
// Pippenger chunks / window trees / tail steps, and the verify pipeline's drain ticks).
//
// ge25519_add (curve25519_ops.cu:326-378) is three dependent product stages — {A, B, T1 T2,
// Z1 Z2} (squares for a doubling), then C = (T1 T2) k, then {E F, G H, F G, E H} — and the four
// products of a stage are independent, so the quad's lanes form one each (operands selected per
// lane) and swap results over DPP: 3 product latencies per operation instead of 9 on one lane.
// Every value is the very product ge_add / ge_dbl forms, so the bits are theirs.  Points are
// replicated over the quad's four lanes on entry and on exit.
#pragma once
#include "ge25519_dev.h"

#ifndef BP_QUAD_SPLITC
#define BP_QUAD_SPLITC 1
#endif
namespace bp {

template <int SRC>
__device__ __forceinline__ uint32_t quad_bcast(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, SRC * 0x55, 0xF, 0xF, true);
}
template <int SRC>
__device__ __forceinline__ fe fe_quad_bcast(const fe& a) {
    fe r;
#pragma unroll
    for (int i = 0; i < 4; i++) {
        uint32_t lo = quad_bcast<SRC>((uint32_t)a.v[i]), hi = quad_bcast<SRC>((uint32_t)(a.v[i] >> 32));
        r.v[i] = (uint64_t)lo | ((uint64_t)hi << 32);
    }
    return r;
}
// (bit masks, not a ternary chain: the compiler turned that into a private array indexed by q,
// i.e. scratch stores and loads inside the dependent chains)
__device__ __forceinline__ fe fe_sel4(int q, const fe& a, const fe& b, const fe& c, const fe& d) {
    const uint64_t m0 = 0ull - (uint64_t)(q & 1), m1 = 0ull - (uint64_t)((q >> 1) & 1);
    fe r;
#pragma unroll
    for (int i = 0; i < 4; i++) {
        const uint64_t ab = a.v[i] ^ ((a.v[i] ^ b.v[i]) & m0), cd = c.v[i] ^ ((c.v[i] ^ d.v[i]) & m0);
        r.v[i] = ab ^ ((ab ^ cd) & m1);
    }
    return r;
}
__device__ __forceinline__ fe fe_sel(bool c, const fe& a, const fe& b) {   // c ? a : b, as masks
    const uint64_t m = 0ull - (uint64_t)c;
    fe r;
#pragma unroll
    for (int i = 0; i < 4; i++) r.v[i] = b.v[i] ^ ((a.v[i] ^ b.v[i]) & m);
    return r;
}

// fe_mul_q4: the product's 64 word products split over the quad by rows — lane rb forms
// (x_{2rb+1} 2^32 + x_{2rb}) * y as an exact 320-bit partial (mul2x8_asm) — and two DPP levels of
// shifted adds sum the partials (the exact 512-bit product) on lane rb = 0, which folds it.
// Valid on the quad's lane 0 only; the same 512 bits as mul512, so the same result bits.
__device__ __forceinline__ uint32_t dpp_qperm_1133(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xF5, 0xF, 0xF, true);   // lane l <- l | 1
}
__device__ __forceinline__ uint32_t dpp_qperm_2222(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xAA, 0xF, 0xF, true);   // lane l <- quad lane 2
}
// this lane's two rows of x: words 2 rb, 2 rb + 1 (rb = the lane's place in its quad)
__device__ __forceinline__ void q4_rows(const fe& x, uint32_t a[2]) {
    const int rb = threadIdx.x & 3;
    const uint64_t m0 = 0ull - (uint64_t)(rb & 1), m1 = 0ull - (uint64_t)((rb >> 1) & 1);
    const uint64_t x01 = x.v[0] ^ ((x.v[0] ^ x.v[1]) & m0), x23 = x.v[2] ^ ((x.v[2] ^ x.v[3]) & m0);
    const uint64_t xr = x01 ^ ((x01 ^ x23) & m1);
    a[0] = (uint32_t)xr;
    a[1] = (uint32_t)(xr >> 32);
}
// the quad's four row partials summed (two DPP levels) and folded on the quad's lane 0
// (BP_Q4_SUM_ASM: the two levels as one list-scheduled asm block, field_asm.h q4_sum_asm: both carry
// chains and the DPP moves interleaved, where the compiled form below waits one state per link)
#ifndef BP_Q4_SUM_ASM
#define BP_Q4_SUM_ASM 1
#endif
template <int LAT = 0>
__device__ __forceinline__ fe fe_q4_sum_fold(const uint32_t w[10], uint32_t* acc = nullptr) {
    uint32_t r[16];
#if BP_Q4_SUM_ASM && defined(__HIP_DEVICE_COMPILE__)
    q4_sum_asm(r, w);
#else
    uint32_t q[12];
    // lanes 0, 2: q = own partial + the next lane's partial at +2 words (12 words)
    uint32_t n1[10];
#pragma unroll
    for (int i = 0; i < 10; i++) n1[i] = dpp_qperm_1133(w[i]);
    unsigned c = 0;
    q[0] = w[0];
    q[1] = w[1];
#pragma unroll
    for (int i = 2; i < 10; i++) q[i] = __builtin_addc(w[i], n1[i - 2], c, &c);
    q[10] = __builtin_addc(n1[8], 0u, c, &c);
    q[11] = n1[9] + c;   // < 2^(32*12) in total: no carry out
    // lane 0: r = q + lane 2's q at +4 words (16 words, the exact 512-bit product)
    uint32_t n2[12];
#pragma unroll
    for (int i = 0; i < 12; i++) n2[i] = dpp_qperm_2222(q[i]);
    c = 0;
#pragma unroll
    for (int i = 0; i < 4; i++) r[i] = q[i];
#pragma unroll
    for (int i = 4; i < 12; i++) r[i] = __builtin_addc(q[i], n2[i - 4], c, &c);
#pragma unroll
    for (int i = 12; i < 15; i++) r[i] = __builtin_addc(n2[i - 4], 0u, c, &c);
    r[15] = n2[11] + c;
#endif
    uint64_t t[8];
#pragma unroll
    for (int i = 0; i < 8; i++) t[i] = (uint64_t)r[2 * i] | ((uint64_t)r[2 * i + 1] << 32);
    return fe_fold512<LAT>(t, acc);
}
template <int LAT = 0>
__device__ __forceinline__ fe fe_mul_q4(const fe& x, const fe& y, uint32_t* acc = nullptr) {
    uint32_t a[2], b[8], w[10];
    q4_rows(x, a);
#pragma unroll
    for (int i = 0; i < 4; i++) {
        b[2 * i] = (uint32_t)y.v[i];
        b[2 * i + 1] = (uint32_t)(y.v[i] >> 32);
    }
    mul2x8_bounded_asm(w, a, b);   // the counting form when a lane's a[0] exceeds the bound (mul512_asm.h)
    if (__builtin_expect(__any(a[0] > MUL_BOUNDED_WORD), 0)) mul2x8_asm(w, a, b);
    return fe_q4_sum_fold<LAT>(w, acc);
}
// fe_mul_q4(x, k) for the curve constant k: the rows by k's SGPR words, one carry counted (mul2x8_k_asm)
template <int LAT = 0>
__device__ __forceinline__ fe fe_mul_q4_k(const fe& x, uint32_t* acc = nullptr) {
    uint32_t a[2], w[10];
    q4_rows(x, a);
    mul2x8_k_asm(w, a);
    return fe_q4_sum_fold<LAT>(w, acc);
}
// Stages 2 and 3 of ge25519_add from the quad's stage-1 products (lane qd holds product qd of
// {A, B, T1 T2, Z1 Z2}); the result replicated over the quad.
__device__ __forceinline__ ge ge_quad_finish(const fe& r1) {
    const int qd = threadIdx.x & 3;
    const fe A = fe_quad_bcast<0>(r1), B = fe_quad_bcast<1>(r1), CT = fe_quad_bcast<2>(r1);
    fe D = fe_quad_bcast<3>(r1);
    const fe C = fe_mul_k(CT);
    D = fe_add(D, D);
    const fe E = fe_sub(B, A), F = fe_sub(D, C), G = fe_add(D, C), H = fe_add(B, A);
    const fe r3 = fe_mul(fe_sel4(qd, E, G, F, E), fe_sel4(qd, F, H, G, H));
    return ge{fe_quad_bcast<0>(r3), fe_quad_bcast<1>(r3), fe_quad_bcast<2>(r3), fe_quad_bcast<3>(r3)};
}

// DBL: add(p, p) (q ignored); else add(p, q).  p, q replicated over the quad; result replicated.
template <bool DBL>
__device__ __forceinline__ ge ge_op_quad(const ge& p, const ge& q) {
    const int qd = threadIdx.x & 3;
    const fe ymx = fe_sub(p.Y, p.X), ypx = fe_add(p.Y, p.X);
    fe r1;
    if (DBL) {
        r1 = fe_sq(fe_sel4(qd, ymx, ypx, p.T, p.Z));
    } else {
        const fe qymx = fe_sub(q.Y, q.X), qypx = fe_add(q.Y, q.X);
        r1 = fe_mul(fe_sel4(qd, ymx, ypx, p.T, p.Z), fe_sel4(qd, qymx, qypx, q.T, q.Z));
    }
    return ge_quad_finish(r1);
}

// A point moved across lane quads of one DPP row: CTRL 0x114 (row_shr:4, lane l takes l-4) or
// 0x104 (row_shl:4, lane l takes l+4).
template <int CTRL>
__device__ __forceinline__ ge ge_row_move(const ge& a) {
    auto mv = [](const fe& f) {
        fe r;
#pragma unroll
        for (int i = 0; i < 4; i++) {
            uint32_t lo = (uint32_t)__builtin_amdgcn_mov_dpp((int)(uint32_t)f.v[i], CTRL, 0xF, 0xF, true);
            uint32_t hi = (uint32_t)__builtin_amdgcn_mov_dpp((int)(uint32_t)(f.v[i] >> 32), CTRL, 0xF, 0xF, true);
            r.v[i] = (uint64_t)lo | ((uint64_t)hi << 32);
        }
        return r;
    };
    return ge{mv(a.X), mv(a.Y), mv(a.Z), mv(a.T)};
}

// ge25519_scalarmult (curve25519_ops.cu:397-415) of one quad: s and P replicated over the quad's
// lanes (quads of one wave may hold different scalars).  The per-lane unified loop of
// sm_lane_loop: every step is one ge25519_add(r, q) with q = r (the doubling) or P, chosen per
// quad; the doubling's stage-1 products are the squares (Y-X)^2, (Y+X)^2, T^2, Z^2 as
// fe_mul(x, x) (== fe_sq(x), the same 512-bit product).  Each lane keeps only its own q-side
// operand of P.  Leading zeros from dtab, or the K-bit prefix table of the base (ptab) as
// scalarmult does; the result replicated over the quad.
//
// Between operations the point is not replicated: each lane keeps only its own stage-1 operand
// ("operand form"), with the lanes' roles chosen so that the stage-3 products land where the next
// stage-1 operands are formed:
//   stage 1   lane 0: A = (Y1-X1)(Y2-X2)   1: T1 T2   2: Z1 Z2   3: B = (Y1+X1)(Y2+X2)
//   stage 3   lane 0: X3 = E F   1: T3 = E H   2: Z3 = G F   3: Y3 = G H   (bit 1 picks G over E,
//             bit 0 H over F: two 2-way selects)
// so T3 and Z3 are already the next T and Z operands, and lanes 0 and 3 swap X3 / Y3 (one DPP
// quad_perm) to form Y3 - X3 and Y3 + X3 (fe_addsub: both chains in one block).  One step: 744 VALU
// and 103 s_nop instead of 808 and 139 (tools/isa_count.py,
// p_quad_step / p_quad_step_of); the products are the same (G F is the integer F G), so the bits.
template <int CTRL>
__device__ __forceinline__ fe fe_dpp(const fe& a) {
    fe r;
#pragma unroll
    for (int i = 0; i < 4; i++) {
        const uint32_t lo = (uint32_t)__builtin_amdgcn_mov_dpp((int)(uint32_t)a.v[i], CTRL, 0xF, 0xF, true);
        const uint32_t hi = (uint32_t)__builtin_amdgcn_mov_dpp((int)(uint32_t)(a.v[i] >> 32), CTRL, 0xF, 0xF, true);
        r.v[i] = (uint64_t)lo | ((uint64_t)hi << 32);
    }
    return r;
}
// p: r in operand form, o = this lane's stage-1 operand; q = this lane's q-side operand (the
// doubling passes o); returns the result's stage-3 product (X3 | T3 | Z3 | Y3 by lane)
template <bool SQ = false>   // SQ: a doubling known to the whole wave (stage 1 as squares, q unused)
__device__ __forceinline__ fe ge_quad_of_step(const fe& o, const fe& q) {
    const int qd = threadIdx.x & 3;
    const fe p1 = SQ ? fe_sq(o) : fe_mul(o, q);
    const fe A = fe_quad_bcast<0>(p1), CT = fe_quad_bcast<1>(p1), D0 = fe_quad_bcast<2>(p1), B = fe_quad_bcast<3>(p1);
#if BP_QUAD_SPLITC   // C = (T1 T2) k split over the quad by rows (fe_mul_q4), then from lane 0 to all
    const fe C = fe_quad_bcast<0>(fe_mul_q4_k(CT));
#else
    const fe C = fe_mul_k(CT);
#endif
    const fe D = fe_add(D0, D0);
    fe E, F, G, H;
    fe_addsub(B, A, H, E);   // H = B + A, E = B - A
    fe_addsub(D, C, G, F);   // G = D + C, F = D - C
    return fe_mul(fe_sel(qd & 2, G, E), fe_sel(qd & 1, H, F));
}
// stage-3 products -> the next operation's operand form (lanes 0 <-> 3 swap: quad_perm [3,1,2,0]):
// lane 0 Y3 - X3, lane 3 Y3 + X3 (= X3 + Y3: the sum and its lossy "- p" are symmetric)
__device__ __forceinline__ fe quad_of_next(const fe& r3) {
    const int qd = threadIdx.x & 3;
    const fe sw = fe_dpp<0x27>(r3);
    fe s, d;
    fe_addsub(sw, r3, s, d);
    return fe_sel(qd == 0, d, fe_sel(qd == 3, s, r3));
}
__device__ __forceinline__ fe quad_of_form(const ge& r) {
    return fe_sel4(threadIdx.x & 3, fe_sub(r.Y, r.X), r.T, r.Z, fe_add(r.Y, r.X));
}
__device__ __forceinline__ ge quad_of_point(const fe& r3) {   // X3 | T3 | Z3 | Y3 -> replicated
    return ge{fe_quad_bcast<0>(r3), fe_quad_bcast<3>(r3), fe_quad_bcast<2>(r3), fe_quad_bcast<1>(r3)};
}
__device__ __forceinline__ ge sm_quad(const fe& s, const ge& P, const ge* __restrict__ dtab, const ge* ptab, int K) {
    const fe qs = quad_of_form(P);
    const int lz = fe_clz256(s);
    const bool pre = K > 0 && lz < K && ptab != nullptr;
    const ge r0 = *(pre ? &ptab[prefix_index(s, K)] : &dtab[lz]);
    int i = pre ? 255 - K : 255 - lz;   // index of the pending bit
    if (i < 0) return r0;
    BitStream bs = bs_init(s, i);
    uint32_t bit = bs_next(bs);
    bool add_phase = false;   // false: next op doubles; true: next op adds P
    fe o = quad_of_form(r0), r3;
    while (true) {
        r3 = ge_quad_of_step(o, fe_sel(add_phase, qs, o));
        if (!add_phase && bit) {
            add_phase = true;
        } else {
            add_phase = false;
            if (--i < 0) break;
            bit = bs_next(bs);
        }
        o = quad_of_next(r3);
    }
    return quad_of_point(r3);
}

// The same on a 16-lane ROW, in operand form: lane quad qi of the row takes role qi of sm_quad's
// lanes (operands Y-X | T | Z | Y+X, stage-3 products X3 | T3 | Z3 | Y3), replicated over its four
// lanes, and every product is split over the quad by rows (fe_mul_q4: four 64 x 256-bit partials,
// two DPP levels, the fold on the quad's lane 0).  A step is then 3 quarter-products deep instead of
// 3 products: for ticks of at most a few thousand items (a one-proof call, a small drain), whose
// time is one scalar-multiplication chain's latency at one wave per SIMD.  The stage results go to
// the row over row_newbcast; quads 0 and 3 swap X3 / Y3 over row_mirror (quad q <-> quad 3 - q;
// the values are replicated over each quad, so the mirrored lane order within a quad is moot).
// The same 512-bit products and the same add / sub / fold code, so the same bits.
template <int SRC>   // lane SRC of each 16-lane row to the whole row (DPP row_newbcast)
__device__ __forceinline__ fe fe_row_bcast(const fe& a) {
    fe r;
#pragma unroll
    for (int i = 0; i < 4; i++) {
        const uint32_t lo = (uint32_t)__builtin_amdgcn_mov_dpp((int)(uint32_t)a.v[i], 0x150 + SRC, 0xF, 0xF, true);
        const uint32_t hi = (uint32_t)__builtin_amdgcn_mov_dpp((int)(uint32_t)(a.v[i] >> 32), 0x150 + SRC, 0xF, 0xF, true);
        r.v[i] = (uint64_t)lo | ((uint64_t)hi << 32);
    }
    return r;
}
// BP_ROW_LAT: the row step's field blocks in their latency forms (field_asm.h *_lat: m = carry | top in
// VALU, no SALU OR waiting on a compare; 2 more VALU per block, which the one wave per SIMD of a row tick
// does not feel)
#ifndef BP_ROW_LAT
#define BP_ROW_LAT 1
#endif
#ifndef BP_ROW_DEFER
#define BP_ROW_DEFER 1
#endif
#ifndef BP_ROW_DEFER_FORCE   // test builds only (tools/ubench_row.hip): every step takes the recompute path
#define BP_ROW_DEFER_FORCE 0
#endif
// LAT 2 (BP_ROW_DEFER): the blocks' fast statements only, their rare-edge words into *acc (sm_row
// recomputes the step with LAT = BP_ROW_LAT when some lane's acc is 2^32-1)
template <int LAT = BP_ROW_LAT>
__device__ __forceinline__ fe ge_row_of_step(const fe& o, const fe& q, uint32_t* acc = nullptr) {
    const int qi = (threadIdx.x >> 2) & 3;
    const fe p1 = fe_mul_q4<LAT>(o, q, acc);   // role qi's stage-1 product, on the quad's lane 0
    const fe A = fe_row_bcast<0>(p1), CT = fe_row_bcast<4>(p1), D0 = fe_row_bcast<8>(p1), B = fe_row_bcast<12>(p1);
    const fe C = fe_quad_bcast<0>(fe_mul_q4_k<LAT>(CT, acc));
    const fe D = fe_add<LAT>(D0, D0, acc);
    fe E, F, G, H;
    fe_addsub<LAT>(B, A, H, E, acc);   // H = B + A, E = B - A
    fe_addsub<LAT>(D, C, G, F, acc);   // G = D + C, F = D - C
    return fe_quad_bcast<0>(fe_mul_q4<LAT>(fe_sel(qi & 2, G, E), fe_sel(qi & 1, H, F), acc));
}
__device__ __forceinline__ fe row_of_next(const fe& r3) {   // quad 0: Y3 - X3, quad 3: X3 + Y3
    const int qi = (threadIdx.x >> 2) & 3;
    const fe sw = fe_dpp<0x140>(r3);   // row_mirror: quad q <- quad 3 - q
    fe s, d;
    fe_addsub<BP_ROW_LAT>(sw, r3, s, d);
    return fe_sel(qi == 0, d, fe_sel(qi == 3, s, r3));
}
__device__ __forceinline__ fe row_of_form(const ge& r) {
    return fe_sel4((threadIdx.x >> 2) & 3, fe_sub(r.Y, r.X), r.T, r.Z, fe_add(r.Y, r.X));
}
__device__ __forceinline__ ge row_of_point(const fe& r3) {   // X3 | T3 | Z3 | Y3 by quad -> replicated
    return ge{fe_row_bcast<0>(r3), fe_row_bcast<12>(r3), fe_row_bcast<8>(r3), fe_row_bcast<4>(r3)};
}
#ifndef BP_ROW_CTRL
#define BP_ROW_CTRL 1
#endif
__device__ __forceinline__ ge sm_row(const fe& s, const ge& P, const ge* __restrict__ dtab, const ge* ptab, int K) {
    const fe qs = row_of_form(P);
    const int lz = fe_clz256(s);
    const bool pre = K > 0 && lz < K && ptab != nullptr;
    const ge r0 = *(pre ? &ptab[prefix_index(s, K)] : &dtab[lz]);
    int i = pre ? 255 - K : 255 - lz;   // index of the pending bit
    if (i < 0) return r0;
    BitStream bs = bs_init(s, i);
    uint32_t bit = bs_next(bs);
    bool add_phase = false;   // false: next op doubles; true: next op adds P
    fe o = row_of_form(r0), r3;
#if BP_ROW_CTRL
    // The same decisions as the branchy loop below, as selects: each 16-lane row has its own scalar,
    // so every per-lane `if` there became an exec-mask save / branch / restore whose SALU half waits
    // on the compare just before it (≈20 cycles each on one wave, tools/ubench_dep.hip).  Here the
    // next op's phase, the bit index and the stream advance are computed before the step (off its
    // critical path), the exit is the one divergent test, and the stream's refill (every 64 bits
    // of a row) runs under a wave-uniform test.
    while (true) {
        const bool take = !add_phase && bit;   // the next op adds P
        const int adv = take ? 0 : 1;           // else: the next bit
        const bool done = i - adv < 0;
        const uint32_t nbit = (uint32_t)(bs.cur >> 63);
#if BP_ROW_DEFER
        {   // one rare-edge test per step instead of one per field block (field_asm.h *_lat_acc)
            const fe qq = fe_sel(add_phase, qs, o);
            uint32_t acc = 0;
            r3 = ge_row_of_step<2>(o, qq, &acc);
            if (BP_ROW_DEFER_FORCE || __builtin_expect(__builtin_amdgcn_ballot_w64(acc == 0xFFFFFFFFu) != 0, 0))
                r3 = ge_row_of_step<BP_ROW_LAT>(o, qq);
        }
#else
        r3 = ge_row_of_step(o, fe_sel(add_phase, qs, o));
#endif
        if (done) break;
        i -= adv;
        add_phase = take;
        bit = adv ? nbit : bit;
        bs.cur = adv ? bs.cur << 1 : bs.cur;
        bs.left -= adv;
        if (__builtin_expect(__builtin_amdgcn_ballot_w64(bs.left == 0) != 0, 0)) {
            const bool rf = bs.left == 0;
            bs.cur = rf ? bs.n1 : bs.cur;
            bs.n1 = rf ? bs.n2 : bs.n1;
            bs.n2 = rf ? bs.n3 : bs.n2;
            bs.n3 = rf ? 0 : bs.n3;
            bs.left = rf ? 64 : bs.left;
        }
        o = row_of_next(r3);
    }
#else
    while (true) {
        r3 = ge_row_of_step(o, fe_sel(add_phase, qs, o));
        if (!add_phase && bit) {
            add_phase = true;
        } else {
            add_phase = false;
            if (--i < 0) break;
            bit = bs_next(bs);
        }
        o = row_of_next(r3);
    }
#endif
    return row_of_point(r3);
}

// The same on a lane PAIR, in operand form: lane 0 holds {Y-X, T}, lane 1 {Y+X, Z}; stage 1: lane 0
// forms A and T1 T2, lane 1 B and Z1 Z2; the pair swaps them over DPP; stage 3: lane 0 X3 = E F and
// T3 = E H, lane 1 Z3 = G F and Y3 = G H (one operand select: G over E on lane 1), so T3 and Z3 are
// already the next operands and the pair swaps X3 / Y3 to form Y3 - X3 / Y3 + X3 (fe_addsub).  5
// product latencies per point operation instead of 9, with 10 products per operation instead of 9
// (a quad forms 12): the form for ticks that fill the SIMDs at two lanes per item but not at four.
__device__ __forceinline__ fe fe_pair_swap(const fe& a) {   // lane l <- lane l ^ 1
    fe r;
#pragma unroll
    for (int i = 0; i < 4; i++) {
        const uint32_t lo = (uint32_t)__builtin_amdgcn_mov_dpp((int)(uint32_t)a.v[i], 0xB1, 0xF, 0xF, true);
        const uint32_t hi = (uint32_t)__builtin_amdgcn_mov_dpp((int)(uint32_t)(a.v[i] >> 32), 0xB1, 0xF, 0xF, true);
        r.v[i] = (uint64_t)lo | ((uint64_t)hi << 32);
    }
    return r;
}
__device__ __forceinline__ void pair_of_form(const ge& r, fe& oa, fe& ob) {
    const bool odd = threadIdx.x & 1;
    fe s, d;
    fe_addsub(r.Y, r.X, s, d);
    oa = fe_sel(odd, s, d);
    ob = fe_sel(odd, r.Z, r.T);
}
// one operation from operand form (oa, ob) with this lane's q-side operands (qa, qb; the doubling
// passes oa, ob): r1 = X3 | Z3, r2 = T3 | Y3
__device__ __forceinline__ void ge_pair_of_step(const fe& oa, const fe& ob, const fe& qa, const fe& qb, fe& r1, fe& r2) {
    const bool odd = threadIdx.x & 1;
    const fe p1 = fe_mul(oa, qa);   // A | B
    const fe p2 = fe_mul(ob, qb);   // T1 T2 | Z1 Z2
    const fe o1 = fe_pair_swap(p1), o2 = fe_pair_swap(p2);
    const fe A = fe_sel(odd, o1, p1), B = fe_sel(odd, p1, o1), CT = fe_sel(odd, o2, p2), D0 = fe_sel(odd, p2, o2);
    const fe C = fe_mul_k(CT);
    const fe D = fe_add(D0, D0);
    fe E, F, G, H;
    fe_addsub(B, A, H, E);
    fe_addsub(D, C, G, F);
    const fe x = fe_sel(odd, G, E);
    r1 = fe_mul(x, F);
    r2 = fe_mul(x, H);
}
__device__ __forceinline__ ge sm_pair(const fe& s, const ge& P, const ge* __restrict__ dtab, const ge* ptab, int K) {
    const bool odd = threadIdx.x & 1;
    fe qa, qb;   // this lane's q-side operands
    pair_of_form(P, qa, qb);
    const int lz = fe_clz256(s);
    const bool pre = K > 0 && lz < K && ptab != nullptr;
    const ge r0 = *(pre ? &ptab[prefix_index(s, K)] : &dtab[lz]);
    int i = pre ? 255 - K : 255 - lz;   // index of the pending bit
    if (i < 0) return r0;
    BitStream bs = bs_init(s, i);
    uint32_t bit = bs_next(bs);
    bool add_phase = false;   // false: next op doubles; true: next op adds P
    fe oa, ob, r1, r2;
    pair_of_form(r0, oa, ob);
    while (true) {
        ge_pair_of_step(oa, ob, fe_sel(add_phase, qa, oa), fe_sel(add_phase, qb, ob), r1, r2);
        if (!add_phase && bit) {
            add_phase = true;
        } else {
            add_phase = false;
            if (--i < 0) break;
            bit = bs_next(bs);
        }
        const fe snd = fe_sel(odd, r2, r1);   // X3 | Y3
        const fe got = fe_pair_swap(snd);      // Y3 | X3
        fe sm, df;
        fe_addsub(got, snd, sm, df);           // lane 0: Y3 - X3; lane 1: X3 + Y3
        oa = fe_sel(odd, sm, df);
        ob = fe_sel(odd, r1, r2);              // T3 | Z3
    }
    const fe s1 = fe_pair_swap(r1), s2 = fe_pair_swap(r2);
    return ge{fe_sel(odd, s1, r1), fe_sel(odd, r2, s2), fe_sel(odd, r1, s1), fe_sel(odd, s2, r2)};
}

}  // namespace bp
