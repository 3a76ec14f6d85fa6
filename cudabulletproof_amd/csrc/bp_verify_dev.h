// bp_verify_dev.h — the verify pipeline's device side: the per-tick task and job functions and the
// k_terms kernel template (one pipeline tick = one launch).  Included by one translation unit per
// tick form (bp_terms1.hip: QL = 1, the throughput form; bp_terms2/4/16.hip: the drain forms), so
// the four large instantiations compile in parallel; bp_kernels.hip holds the other verify kernels.
#pragma once
#include "bp_kernels.h"
#include "ge25519_dev.h"
#include "ge25519_quad.h"
#include "sha256_dev.h"

namespace bp {

#ifndef BP_TERMS_OCC
#define BP_TERMS_OCC 4   // k_terms blocks per CU the register budget is sized for
#endif
constexpr int TPB = 256;   // threads per k_terms block (bp_kernels.hip, which does not include this header, has its own)
__device__ __forceinline__ size_t gid() { return (size_t)blockIdx.x * blockDim.x + threadIdx.x; }

// ------------------------------------------------------------------ verify: challenges & scalars


// range_proof_verify's scalar work (mode 2), one lane per proof: the x challenge
// (challenge.cu:61-77), compute_precise_delta (rp.cu:315-410), enhanced_range_check
// (rp.cu:765-876; called twice at rp.cu:1778/:1785 with the same result), the V match
// (rp.cu:1729-1740) and the polynomial-identity scalars in host-tobytes form (rp.cu:424-435).
// sy = <1^n, y^n> from the caller's power loop (rp.cu:336-343, the same mul/add chain).
__device__ __forceinline__ void prep_std_task(const BatchView& bv, const VerifyWs& ws, const fe* __restrict__ two_i,
                                              size_t p, const fe& z, const fe& z2, const fe& sy) {
    const int n = bv.n;
    fe x = chal_x(bv.T1[p], bv.T2[p]);   // 4 bytes of "xchal" (challenge.cu:73)
    const fe two = fe_add(fe_set(1), fe_set(1));
    // compute_precise_delta
    fe z3 = fe_mul(z2, z);
    fe t1 = fe_mul(fe_sub(z, z2), sy);
    fe s2 = fe_set(1);
    for (int i = 1; i < n; i++) s2 = fe_add(s2, two_i[i]);   // sum of 2^i, two_i[i] = the i-fold mul chain
    fe delta = fe_sub(t1, fe_mul(z3, s2));
    // enhanced_range_check
    const fe t = bv.t[p];
    fe tmd = fe_sub(t, delta);
    fe val = fe_mul(tmd, fe_invert(z2));
    fe two_n = fe_mul(two_i[n - 1], two);                    // n-fold mul chain from 1
    bool lower_ok = (fe_canon(fe_sub(tmd, z2)).v[3] >> 63) == 0;
    bool upper_ok = (fe_canon(fe_sub(fe_mul(z2, two_n), tmd)).v[3] >> 63) == 0;
    fe dm = fe_canon(fe_sub(val, two_n));
    bool close = true;
    for (int i = 0; i < 4; i++) {
        uint32_t b = fe_byte(dm, i);
        close &= !(b > 3 && b < 253);
    }
    bool range_ok = lower_ok & upper_ok & !close;
    const ge& Vp = bv.Vp ? bv.Vp[p] : bv.V[p];
    bool vmatch = fe_eq(fe_canon(bv.V[p].X), fe_canon(Vp.X)) & fe_eq(fe_canon(bv.V[p].Y), fe_canon(Vp.Y));
    ws.rflags[p] = (uint8_t)((vmatch ? 1 : 0) | (range_ok ? 2 : 0));
    ws.pbase[p * 3 + 0] = bv.V[p];
    ws.pbase[p * 3 + 1] = bv.T1[p];
    ws.pbase[p * 3 + 2] = bv.T2[p];
    fe* ps = ws.psc + p * 8;
    ps[0] = fe_canon(t);
    ps[1] = fe_canon(bv.taux[p]);
    ps[2] = fe_canon(z2);
    ps[3] = fe_canon(delta);
    ps[4] = fe_canon(bv.mu[p]);
    ps[5] = fe_canon(x);
    ps[6] = fe_canon(fe_mul(x, x));
}

// cuda_range_proof_verify (crv:93-106) + calculate_inner_product_point scalars
// (bulletproof_range_proof.cu:679-718): one lane per proof.
__device__ __forceinline__ void prep_range_task(const BatchView& bv, const VerifyWs& ws, const fe* __restrict__ two_i,
                                             size_t p, int mode) {
    const int n = bv.n;
    // y = H("BulletproofYChal" || V.X V.Y A.X A.Y S.X S.Y || "y_ch")   (challenge.cu:24-44)
    fe y = chal_y(bv.V[p], bv.A[p], bv.S[p]);
    // z = H("BulletproofZChal" || y || "z_ch")   (challenge.cu:47-58)
    fe z = chal_z(y);
    // (x is derived at crv:105 but only feeds compute_precise_delta and the unused
    //  x argument of calculate_inner_product_point; it does not affect any output.)
    fe z2 = fe_mul(z, z);
    ws.sG[p] = fe_sub(fe_set(0), z);   // rp.cu:699  0 - z
    fe pw = fe_set(1), sy = fe_set(1);
    for (int i = 0; i < n; i++) {
        if (i > 0) {
            pw = fe_mul(pw, y);          // powers_of (rp.cu:299-313)
            sy = fe_add(sy, pw);         // <1^n, y^n> (rp.cu:341-342), mode 2 only
        }
        fe h = fe_add(z, fe_mul(z2, two_i[i]));
        ws.sH[p * n + i] = fe_mul(h, pw);
    }
    ws.sc[p * 4 + 0] = fe_canon(bv.t[p]);
    if (mode == 2) prep_std_task(bv, ws, two_i, p, z, z2, sy);
}

// cuda_inner_product_verify (crv:146-218): <a,b> check and the per-round challenges.
__device__ __forceinline__ void prep_ipa_task(const BatchView& bv, const VerifyWs& ws, size_t p) {
    const int abl = bv.ab_len, Lr = bv.L_len;
    fe acc = fe_set(0);
    for (int i = 0; i < abl; i++) acc = fe_add(acc, fe_mul(bv.a[p * abl + i], bv.b[p * abl + i]));   // vectors.cu:101
    ws.ipok[p] = fe_eq(fe_canon(acc), fe_canon(bv.c[p])) ? 1 : 0;
    fe tr = fe_set(0);   // transcript (crv:168)
    for (int r = 0; r < Lr; r++) {
        fe u;
        if (r == 0) {
            u = bv.x[p];
        } else {
            u = chal_ip(tr, bv.L[p * Lr + r].X, bv.R[p * Lr + r].X);
            tr = u;
        }
        ws.u[p * Lr + r] = fe_canon(u);
        ws.uinv[p * Lr + r] = fe_canon(fe_invert(u));
    }
    ws.sc[p * 4 + 1] = fe_canon(bv.a[p * abl]);
    ws.sc[p * 4 + 2] = fe_canon(bv.b[p * abl]);
    ws.sc[p * 4 + 3] = fe_canon(bv.c[p]);
}

// The drain forms' challenge region (QL >= 4: a tick of a few thousand proofs at most, whose time is
// the length of these per-proof chains): each proof on a lane quad, lane qd = threadIdx.x & 3.  The
// sequential parts (the hashes, the y-power chain, the transcript) run on all four lanes alike; the
// independent products of each group of four indices and the round challenges' inversions are
// spread over the lanes.  The same operations on the same values, so the same bits as
// prep_range_task / prep_ipa_task.
__device__ __forceinline__ void prep_range_task_q4(const BatchView& bv, const VerifyWs& ws,
                                                   const fe* __restrict__ two_i, size_t p, int mode, int qd) {
    const int n = bv.n;
    const fe y = chal_y(bv.V[p], bv.A[p], bv.S[p]);
    const fe z = chal_z(y);
    const fe z2 = fe_mul(z, z);
    if (qd == 0) ws.sG[p] = fe_sub(fe_set(0), z);
    fe pw = fe_set(1), sy = fe_set(1), mine = fe_set(1);
    for (int i0 = 0; i0 < n; i0 += 4) {
#pragma unroll
        for (int j = 0; j < 4; j++) {   // powers i0 .. i0 + 3 (wave-uniform), lane qd keeps power i0 + qd
            const int i = i0 + j;
            if (i > 0 && i < n) {
                pw = fe_mul(pw, y);
                sy = fe_add(sy, pw);
            }
            mine = fe_sel(j == qd, pw, mine);
        }
        const int i = i0 + qd;
        if (i < n) ws.sH[p * n + i] = fe_mul(fe_add(z, fe_mul(z2, two_i[i])), mine);
    }
    if (qd == 0) {
        ws.sc[p * 4 + 0] = fe_canon(bv.t[p]);
        if (mode == 2) prep_std_task(bv, ws, two_i, p, z, z2, sy);
    }
}

__device__ __forceinline__ void prep_ipa_task_q4(const BatchView& bv, const VerifyWs& ws, size_t p, int qd) {
    const int abl = bv.ab_len, Lr = bv.L_len;
    if (Lr > 16) {   // (more rounds than four registers per lane hold: the one-lane form)
        if (qd == 0) prep_ipa_task(bv, ws, p);
        return;
    }
    fe acc = fe_set(0);
    for (int i = 0; i < abl; i++) acc = fe_add(acc, fe_mul(bv.a[p * abl + i], bv.b[p * abl + i]));
    fe tr = fe_set(0), m0 = tr, m1 = tr, m2 = tr, m3 = tr;   // lane qd: u_r for r = qd, 4 + qd, ...
    for (int r = 0; r < Lr; r++) {
        fe u;
        if (r == 0) {
            u = bv.x[p];
        } else {
            u = chal_ip(tr, bv.L[p * Lr + r].X, bv.R[p * Lr + r].X);
            tr = u;
        }
        const bool me = (r & 3) == qd;
        const int k = r >> 2;
        m0 = fe_sel(me && k == 0, u, m0);
        m1 = fe_sel(me && k == 1, u, m1);
        m2 = fe_sel(me && k == 2, u, m2);
        m3 = fe_sel(me && k == 3, u, m3);
    }
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const int r = 4 * k + qd;
        const fe u = k == 0 ? m0 : k == 1 ? m1 : k == 2 ? m2 : m3;
        if (r < Lr) {
            ws.u[p * Lr + r] = fe_canon(u);
            ws.uinv[p * Lr + r] = fe_canon(fe_invert(u));
        }
    }
    if (qd == 0) {
        ws.ipok[p] = fe_eq(fe_canon(acc), fe_canon(bv.c[p])) ? 1 : 0;
        ws.sc[p * 4 + 1] = fe_canon(bv.a[p * abl]);
        ws.sc[p * 4 + 2] = fe_canon(bv.b[p * abl]);
        ws.sc[p * 4 + 3] = fe_canon(bv.c[p]);
    }
}

// ------------------------------------------------------------------ verify: scalar multiplications
// IPA fold round r (crv:220-242), n' = n >> (r+1).  Items per proof (4n'):
//   [0,n')   u^-1 * G_j        [n',2n')  u^-1 * H_{j+n'}
//   [2n',3n') u * G_{j+n'}     [3n',4n') u * H_j
// (lanes sharing a scalar are adjacent).  Round 0 reads the generators; round r >= 1 reads
// the folded G'/H' of round r-1, each of which exactly one item of round r consumes, so the
// item forms it itself from the two round r-1 terms (crv:230, :240):
//   G'_m = N(term(u^-1 G_m) + term(u G_{m+n''})),  H'_m = N(term(u H_m) + term(u^-1 H_{m+n''}))
// with n'' = 2n' and the round r-1 terms at fold[(r-1) & 1] in the item order above.
__device__ __forceinline__ ge folded_point(const VerifyWs& ws, int n, int r, size_t p, bool isH, int m) {
    const int npp = n >> r;   // n'' = the previous round's n'
    const ge* f = ws.fold[(r - 1) & 1] + p * (2 * n);
    if (!isH) return ge_norm_host(ge_add(f[m], f[2 * npp + m]));
    return ge_norm_host(ge_add(f[3 * npp + m], f[npp + m]));
}

// One scalar multiplication of a tick: its scalar, its point, where the result goes and which
// normalize it gets.  Every task kind only FILLS a job; k_terms then runs the one scalarmult call
// site for all of them, so the launch carries one copy of the scalar-mult loops instead of one per
// task kind (each copy is tens of KB of straight-line code: several copies live in one launch
// thrash the instruction cache of CUs running waves of different kinds).
struct SmJob {
    fe s;
    ge P;
    ge* dst;
    int dev_norm;   // 1: device normalize (MSM terms, kernels.cu:26-42), 0: host normalize
    int base;       // the fixed base's prefix-table row (SlotDev::ptab), -1: none
};

// Lane and item indices of a tick are 32-bit (the host keeps a launch below 2^32 lanes) and n
// is a power of two: index arithmetic is shifts and masks, no 64-bit division sequences.
// (log2n: bp_kernels.h)

__device__ __forceinline__ void fold_job(const BatchView& bv, const VerifyWs& ws, int r, uint32_t p, uint32_t k,
                                         const ge* __restrict__ G, const ge* __restrict__ H, SmJob& jb) {
    const int n = bv.n, lnp = log2n(n) - r - 1, np = 1 << lnp, Lr = bv.L_len;   // np = n >> (r + 1)
    const int grp = (int)(k >> lnp), j = (int)(k & (np - 1));
    const bool isH = grp == 1 || grp == 3;
    const int m = (grp == 1 || grp == 2) ? j + np : j;
    jb.s = (grp < 2) ? ws.uinv[(size_t)p * Lr + r] : ws.u[(size_t)p * Lr + r];
    if (r == 0) {
        jb.P = isH ? H[m] : G[m];
        jb.base = isH ? n + m : m;
    } else {
        jb.P = folded_point(ws, n, r, p, isH, m);
    }
    jb.dst = ws.fold[r & 1] + (size_t)p * (2 * n) + k;
    jb.dev_norm = 0;
}

// (stage0_class_item / stage0_item: bp_kernels.h, host-checked by tests/host_lanes_check.hip)

// Stage 0: every scalar multiplication that depends only on the proof.  Item index space
// (lanes reach it through stage0_item's class layout):
//   [0, 2nB)      the two MSMs of calculate_inner_product_point (rp.cu:724, :728):
//                 segment 2p = <sG, G>, 2p+1 = <sH, H>; Ndev (kernels.cu:26-42)
//   [.., +2nB)    IPA fold round 0 terms
//   [.., +2B)     t*h (rp.cu:778-781) and c*Q (crv:255, :268-269), host normalize
//   [.., +7B)     mode 2: the polynomial identity's g^t, h^taux, V^z^2, g^delta, h^mu, T1^x, T2^x^2
//                 (rp.cu:442-480), host normalize

__device__ __forceinline__ bool stage0_job(const SlotDev& sd, uint32_t i, const ge* __restrict__ G,
                                          const ge* __restrict__ H, const ge* __restrict__ g,
                                          const ge* __restrict__ h, SmJob& jb) {
    const BatchView& bv = sd.bv;
    const VerifyWs& ws = sd.ws;
    const uint32_t B = (uint32_t)bv.B;
    const int n = bv.n, ln = log2n(n);
    const uint32_t nA = sd.range_mode ? B << (ln + 1) : 0;
    const uint32_t nB = bv.L_len > 0 ? B << (ln + 1) : 0;
    if (i < nA) {
        const uint32_t seg = i >> ln;
        const int k = (int)(i & (n - 1));
        const uint32_t p = seg >> 1;
        const bool isH = seg & 1;
        jb.s = isH ? ws.sH[(size_t)p * n + k] : ws.sG[p];
        jb.P = isH ? H[k] : G[k];
        jb.base = isH ? n + k : k;
        jb.dst = ws.msm_pts + i;
        jb.dev_norm = 1;
        return true;
    }
    i -= nA;
    if (i < nB) {
        fold_job(bv, ws, 0, i >> (ln + 1), i & (2 * n - 1), G, H, jb);
        return true;
    }
    i -= nB;
    if (i < 2 * B) {
        const uint32_t p = i >> 1;
        const bool isC = i & 1;
        if (!isC && !sd.range_mode) return false;
        jb.s = isC ? ws.sc[(size_t)p * 4 + 3] : ws.sc[(size_t)p * 4 + 0];
        jb.P = *h;
        jb.base = 2 * n;
        jb.dst = ws.terms + (size_t)p * 4 + 2 + (isC ? 1 : 0);
        jb.dev_norm = 0;
        return true;
    }
    i -= 2 * B;
    const uint32_t p = i / 7u;
    const int k = (int)(i - 7u * p);
    if (k == 0 || k == 3) { jb.P = *g; jb.base = 2 * n + 1; }
    else if (k == 1 || k == 4) { jb.P = *h; jb.base = 2 * n; }
    else if (k == 2) jb.P = ws.pbase[(size_t)p * 3 + 0];
    else if (k == 5) jb.P = ws.pbase[(size_t)p * 3 + 1];
    else jb.P = ws.pbase[(size_t)p * 3 + 2];
    jb.s = ws.psc[(size_t)p * 8 + k];
    jb.dst = ws.pterm + (size_t)p * 8 + k;
    jb.dev_norm = 0;
    return true;
}

// range_proof_verify method 3 (rp.cu:568-580): chal * left, chal * right, host normalize.
// The scalar is the raw SHA-256 digest bytes.  Items: 2p -> left, 2p+1 -> right.
__device__ __forceinline__ void m3_job(const SlotDev& sd, uint32_t i, SmJob& jb) {
    jb.s = sd.ws.chal[i >> 1];
    jb.P = sd.ws.lr[i];
    jb.dst = sd.ws.m3 + i;
    jb.dev_norm = 0;
}

// a0*G'_0 and b0*H'_0 (crv:262-266).  Items: 2p -> a0*G', 2p+1 -> b0*H'.
__device__ __forceinline__ void final_terms_job(const SlotDev& sd, uint32_t i, const ge* __restrict__ G,
                                                const ge* __restrict__ H, SmJob& jb) {
    const BatchView& bv = sd.bv;
    const VerifyWs& ws = sd.ws;
    const uint32_t p = i >> 1;
    bool isH = i & 1;
    const int n = bv.n;
    jb.s = ws.sc[(size_t)p * 4 + (isH ? 2 : 1)];
    // G'_0 / H'_0 after the last round (formed from its terms), the generators when there is none
    if (bv.L_len > 0) jb.P = folded_point(ws, n, bv.L_len, p, isH, 0);
    else jb.P = isH ? H[0] : G[0];
    jb.dst = ws.fin + (size_t)p * 2 + (isH ? 1 : 0);
    jb.dev_norm = 0;
}

// Region lookup with constant indices only (a run-time index into the by-value kernel
// argument would copy the whole list to scratch).
__device__ __forceinline__ Region find_region(const RegionList& rl, size_t i) {
    Region g = rl.reg[0];
#pragma unroll
    for (int k = 1; k < MAX_REGIONS; k++)
        if (k < rl.count && i >= rl.reg[k].begin) g = rl.reg[k];
    return g;
}

__device__ __forceinline__ int absdiff(int a, int b) { return a > b ? a - b : b - a; }

// Canonical MSM tree over cnt points stored `stride` apart, evaluated level by
// level by one lane, in place (the slot's own workspace): stride 1 = the whole tree of an
// n <= LANE_TREE_MAX MSM; stride TPB = levels TPB, 2 TPB, ... over the per-block chunk roots.
// QUAD (drain ticks): the proof's lane quad runs each add on ge_op_quad (3 product latencies
// instead of 9); all four lanes hold and store the same values, so each reads back its own writes.
template <bool QUAD = false>
__device__ __forceinline__ ge gadd(const ge& a, const ge& b) {
    if (QUAD) return ge_op_quad<false>(a, b);
    return ge_add(a, b);
}
template <bool QUAD = false>
__device__ __forceinline__ ge tree_upper(ge* T, int cnt, int stride) {
    for (int st = 1; st < cnt; st <<= 1)
        for (int i = 0; i + st < cnt; i += 2 * st)
            T[(size_t)i * stride] = ge_norm_dev(gadd<QUAD>(T[(size_t)i * stride], T[(size_t)(i + st) * stride]));
    return T[0];
}

// P assembly (rp.cu:785-801), check point (crv:257-278) and the tolerant accept rule
// (crv:297-357).  One lane per proof; QUAD: one lane quad per proof (its point adds on the quad,
// the rest computed alike by the four lanes, lane 0 of the quad writes the outputs).
template <bool QUAD = false>
__device__ __forceinline__ void final_task(const SlotDev& sd, size_t p) {
    const bool wr = !QUAD || (threadIdx.x & 3) == 0;
    const VerifyWs& ws = sd.ws;
    ge P;
    if (sd.range_mode) {
        ge m0, m1;
        const int n = sd.bv.n;
        if (!sd.lane_tree && n > TPB) {   // upper tree levels over the per-block chunk roots (RK_TREE)
            m0 = tree_upper<QUAD>(ws.msm_pts + (p * 2 + 0) * n, n / TPB, TPB);
            m1 = tree_upper<QUAD>(ws.msm_pts + (p * 2 + 1) * n, n / TPB, TPB);
        } else {                    // RK_LTREE (whole lane trees, any n) or RK_TREE blocks (n <= TPB) wrote them
            m0 = ws.msm_part[p * 2 + 0];
            m1 = ws.msm_part[p * 2 + 1];
        }
        P = ge_zero();
        P = ge_norm_host(gadd<QUAD>(P, m0));
        P = ge_norm_host(gadd<QUAD>(P, m1));
        P = ge_norm_host(gadd<QUAD>(P, ws.terms[p * 4 + 2]));
        P = ge_norm_host(P);
        P = ge_norm_host(P);
    } else {
        P = ws.Pin[p];
    }
    ge cp = ge_zero();
    cp = ge_norm_host(gadd<QUAD>(cp, ws.fin[p * 2 + 0]));
    cp = ge_norm_host(gadd<QUAD>(cp, ws.fin[p * 2 + 1]));
    cp = ge_norm_host(gadd<QUAD>(cp, ws.terms[p * 4 + 3]));
    if (wr && sd.P_out) sd.P_out[p] = P;
    if (wr && sd.chk_out) sd.chk_out[p] = cp;

    fe kx = fe_canon(cp.X), ky = fe_canon(cp.Y), px = fe_canon(P.X), py = fe_canon(P.Y);
    if (sd.range_mode == 2) {
        // range_proof_verify (rp.cu:1717-1815): V match && range check && polynomial identity
        // && inner_product_verify, whose accept rule is vectors.cu:713-749 on X bytes.
        const uint8_t fl = ws.rflags[p];
        fe lmx = fe_canon(ws.m3[p * 2].X), rmx = fe_canon(ws.m3[p * 2 + 1].X);
        int tot = 0;
        for (int i = 0; i < 4; i++) tot += 64 - __popcll(lmx.v[i] ^ rmx.v[i]);
        int top = 64 - __popcll(lmx.v[3] ^ rmx.v[3]);           // bytes 24..31 (rp.cu:595-601)
        bool m3 = top >= 22, m4 = tot >= 200;                     // rp.cu:606-627
        bool poly_ok = ((fl >> 2) & 1) | m3 | m4;
        int xdc = 0, sxc = 0;
        for (int i = 0; i < 32; i++) {
            int d = absdiff((int)fe_byte(kx, i), (int)fe_byte(px, i));
            xdc += d > 0;
            sxc += (d > 0) & (d <= 5);
        }
        int mb = 64 - __popcll(kx.v[3] ^ px.v[3]);
        bool ip_ok = ws.ipok[p] && ((xdc <= 3) | (sxc >= 28) | (mb >= 20));
        if (!wr) return;
        sd.ok[p] = ((fl & 1) && ((fl >> 1) & 1) && poly_ok && ip_ok) ? 1 : 0;
        if (sd.flags_out)
            sd.flags_out[p] = (uint8_t)((fl & 7) | (m3 ? 8 : 0) | (m4 ? 16 : 0) | (ip_ok ? 32 : 0));
        if (sd.poly_out) {
            sd.poly_out[p * 4 + 2] = ws.m3[p * 2];
            sd.poly_out[p * 4 + 3] = ws.m3[p * 2 + 1];
        }
        return;
    }
    int xd = 0, yd = 0, sx = 0, sy = 0, msb = 0;
    for (int i = 0; i < 32; i++) {
        int a = (int)((kx.v[i >> 3] >> (8 * (i & 7))) & 0xff), b = (int)((px.v[i >> 3] >> (8 * (i & 7))) & 0xff);
        int c2 = (int)((ky.v[i >> 3] >> (8 * (i & 7))) & 0xff), d = (int)((py.v[i >> 3] >> (8 * (i & 7))) & 0xff);
        int dx = absdiff(a, b), dy = absdiff(c2, d);
        xd += dx > 0; yd += dy > 0;
        sx += (dx > 0) & (dx <= 10); sy += (dy > 0) & (dy <= 10);
    }
    msb = 64 - __popcll(kx.v[3] ^ px.v[3]);   // bits of bytes 24..31 of X
    const fe hs = sha_4fe(kx, ky, px, py);
    int hz = 0;
    for (int i = 0; i < 32; i++) hz += ((hs.v[i >> 3] >> (8 * (i & 7))) & 0xff) != 0;
    bool accept = (sx + sy >= 20) | (msb >= 28) | (xd + yd <= 32) | (hz <= 24);
    if (wr) sd.ok[p] = (ws.ipok[p] && accept) ? 1 : 0;
}

// The two MSMs' canonical trees of a proof whose MSMs have n <= LANE_TREE_MAX points (RK_LTREE):
// every add with all lanes busy; QUAD (drain ticks): on the proof's lane quad.
template <bool QUAD>
__device__ __forceinline__ void ltree_task(const SlotDev& sd, size_t p) {
    const VerifyWs& ws = sd.ws;
    const int n = sd.bv.n;
    const ge m0 = tree_upper<QUAD>(ws.msm_pts + (p * 2 + 0) * n, n, 1);
    const ge m1 = tree_upper<QUAD>(ws.msm_pts + (p * 2 + 1) * n, n, 1);
    if (!QUAD || (threadIdx.x & 3) == 0) {
        ws.msm_part[p * 2 + 0] = m0;
        ws.msm_part[p * 2 + 1] = m1;
    }
}

// range_proof_verify's polynomial identity sides and methods 1-2 (rp.cu:452-530), then the
// method-3 challenge SHA-256(left.X | left.Y | right.X | right.Y) (rp.cu:560-566).  One lane per proof.
__device__ __forceinline__ void poly_task(const SlotDev& sd, size_t p) {
    const VerifyWs& ws = sd.ws;
    const ge* t = ws.pterm + p * 8;
    ge left = ge_norm_host(ge_add(t[0], t[1]));
    ge right = ge_zero();
    for (int k = 2; k < 7; k++) right = ge_norm_host(ge_add(right, t[k]));
    left = ge_norm_host(left);
    right = ge_norm_host(right);
    fe lx = fe_canon(left.X), ly = fe_canon(left.Y), rx = fe_canon(right.X), ry = fe_canon(right.Y);
    int dxc = 0, dyc = 0, sxc = 0, syc = 0, cons = 0, prev = 0;
    bool est = false;
    for (int i = 0; i < 32; i++) {
        int a = (int)fe_byte(lx, i), b = (int)fe_byte(rx, i);
        int xd = absdiff(a, b), yd = absdiff((int)fe_byte(ly, i), (int)fe_byte(ry, i));
        dxc += xd > 0; dyc += yd > 0;
        sxc += (xd > 0) & (xd <= 10); syc += (yd > 0) & (yd <= 10);
        int diff = a - b;
        if (!est && diff != 0) {
            prev = diff;
            est = true;
        } else if (est && absdiff(diff, prev) <= 10) {
            cons++;
            prev = (prev * 3 + diff) / 4;   // C division: truncation toward zero
        }
    }
    (void)dyc;
    bool m12 = (dxc <= 5) | ((sxc >= 24) & (syc >= 20)) | (cons >= 20);
    const fe ch = sha_4fe(lx, ly, rx, ry);
    ws.chal[p] = ch;
    ws.lr[p * 2] = left;
    ws.lr[p * 2 + 1] = right;
    ws.rflags[p] |= m12 ? 4 : 0;
    if (sd.poly_out) {
        sd.poly_out[p * 4] = left;
        sd.poly_out[p * 4 + 1] = right;
    }
}

// One pipeline tick = ONE launch.  Every region is one in-flight batch at its own stage
// (challenges / stage 0 / MSM trees / fold round r / final terms / final assembly), so a launch
// carries a whole batch's worth of independent work however deep the batch-level dependency
// chain is, and the short per-proof chains (trees, final assembly) run under the scalar
// multiplications of the other batches instead of in a latency-bound launch of their own.
// The RK_TREE region (if any) comes first and spans whole blocks: each block folds TPB/n
// segments of the batch's 2B MSMs with the canonical tree of k_tree, barriers block-uniform;
// its LDS is the q-operand array (no scalar multiplication runs in those blocks).
//
// QL = lanes per scalar-multiplication item (Pipeline::push picks it per tick): 1 the throughput
// form; 4 (the drain ticks, too small to fill the SIMDs, whose time is one scalar-multiplication
// chain's latency) a lane quad per item running sm_quad, 3 product latencies per point operation
// instead of 9, and the chains (RK_LTREE, RK_FINAL) on quads too; 2 a lane pair per item running
// sm_pair (5 product latencies, 10 products instead of 9), for ticks between the two; 16 (the
// smallest ticks: a one-proof call) a 16-lane row per item running sm_row, each product split
// over a quad, the chains on quads.  Region items are QL lanes each (chains 4 in the row form).
// The same operations in every form, so the same bits.
// The drain forms (QL >= 2) run ticks of at most 65,536 lanes, i.e. at most about one wave per SIMD:
// they get the register budget of BP_DRAIN_OCC blocks per CU (256 VGPRs at 2) instead of the
// throughput form's 128, so their chains (challenges, assembly, lane trees) compile without spills.
#ifndef BP_DRAIN_OCC
#define BP_DRAIN_OCC 2
#endif
#ifdef BP_TERMS_WPE   // A/B: a register budget for more waves per SIMD than k_terms runs (room for other kernels' waves)
#define BP_TERMS_BOUNDS(QL) __launch_bounds__(TPB) __attribute__((amdgpu_waves_per_eu(BP_TERMS_WPE, 8)))
#else
#define BP_TERMS_BOUNDS(QL) __launch_bounds__(TPB, (QL) >= 2 ? BP_DRAIN_OCC : BP_TERMS_OCC)
#endif
template <int QL>
__global__ BP_TERMS_BOUNDS(QL) void k_terms(RegionList rl, const SlotDev* __restrict__ slots,
                                               const ge* __restrict__ G, const ge* __restrict__ H,
                                               const ge* __restrict__ g, const ge* __restrict__ h,
                                               const ge* __restrict__ dtab, const fe* __restrict__ two_i) {
    __shared__ geq qs[TPB];
    size_t i = gid();
    if (i >= rl.total) return;
    const Region rg = find_region(rl, i);
    size_t l = i - rg.begin;
    const SlotDev& sd = slots[rg.slot];
    if (rg.kind == RK_TREE) {
        // chunks of min(n, TPB) points: n <= TPB -> one MSM per chunk, root to msm_part;
        // n > TPB -> the chunk root is written back in place at the chunk's first point and
        // final_task runs the remaining levels (tree_upper).
        ge* sh = reinterpret_cast<ge*>(qs);
        const int n = sd.bv.n, ch = n < TPB ? n : TPB, tid = threadIdx.x, idx = tid & (ch - 1);
        const bool live = l < rg.items;   // a whole chunk is live or not (items: a multiple of ch)
        if (live) sh[tid] = sd.ws.msm_pts[l];
        __syncthreads();
        for (int st = 1; st < ch; st <<= 1) {   // pairs packed onto the chunk's first lanes (k_tree)
            const int j = tid - idx + 2 * st * idx;
            if (live && 2 * st * idx + st < ch) sh[j] = ge_norm_dev(ge_add(sh[j], sh[j + st]));
            __syncthreads();
        }
        if (live && idx == 0) {
            if (n <= TPB) sd.ws.msm_part[l / n] = sh[tid];
            else sd.ws.msm_pts[l] = sh[tid];
        }
        return;
    }
    if (l >= rg.items) return;
    if (rg.kind == RK_PREP) {
        // lanes [0,B): range-proof challenges and MSM scalars (range mode only), then [.., +B): IPA
        const size_t B = sd.bv.B;
        if (QL >= 4) {   // a lane quad per proof (region_lanes)
            const size_t it = l >> 2;
            const int qd = threadIdx.x & 3;
            if (sd.range_mode && it < B) prep_range_task_q4(sd.bv, sd.ws, two_i, it, sd.range_mode, qd);
            else prep_ipa_task_q4(sd.bv, sd.ws, sd.range_mode ? it - B : it, qd);
        } else if (sd.range_mode && l < B) {
            prep_range_task(sd.bv, sd.ws, two_i, l, sd.range_mode);
        } else {
            prep_ipa_task(sd.bv, sd.ws, sd.range_mode ? l - B : l);
        }
    } else if (rg.kind == RK_POLY) {
        poly_task(sd, l);
    } else if (rg.kind == RK_FINAL) {
        if (QL >= 4) final_task<true>(sd, l >> 2);   // the chains stay on quads in the row form
        else final_task<false>(sd, l);
    } else if (rg.kind == RK_LTREE) {
        if (QL >= 4) ltree_task<true>(sd, l >> 2);
        else ltree_task<false>(sd, l);
    } else {
        // the scalar-multiplication kinds: fill the job, then the one call site
        SmJob jb;
        jb.base = -1;
        bool live = true;
        uint32_t li = (uint32_t)l;   // < 2^32: Pipeline::push keeps a tick below 2^32 lanes
        if (QL == 16) li >>= 4;      // the row's / quad's / pair's item
        if (QL == 4) li >>= 2;
        if (QL == 2) li >>= 1;
        if (rg.kind == RK_STAGE0 || rg.kind == RK_MSMT) {
            // RK_MSMT: a chunk of the split stage 0's second part, lanes from rg.r on
            const uint32_t it = rg.kind == RK_MSMT ? stage0_item(sd, (uint32_t)rg.r + li, S0_DEFER)
                                                   : stage0_item(sd, li, sd.defer ? S0_CRIT : S0_ALL);
            live = it != UINT32_MAX && stage0_job(sd, it, G, H, g, h, jb);
        } else if (rg.kind == RK_M3) {
            m3_job(sd, li, jb);
        } else if (rg.kind == RK_ROUND) {
            const int l4 = log2n(sd.bv.n) - rg.r + 1;   // 4 n' = 2^l4 items per proof
            if (const uint32_t* pm = sd.permr[rg.r]) li = pm[li];
            fold_job(sd.bv, sd.ws, rg.r, li >> l4, li & ((1u << l4) - 1), G, H, jb);
        } else {   // RK_FINAL_TERMS
            if (sd.perm_ft) li = sd.perm_ft[li];
            final_terms_job(sd, li, G, H, jb);
        }
        if (live) {
            const ge* pt = (sd.ptab && jb.base >= 0) ? sd.ptab + ((size_t)jb.base << sd.pbits) : nullptr;
            if (QL == 16) {
                const ge t = sm_row(jb.s, jb.P, dtab, pt, pt ? sd.pbits : 0);
                if ((threadIdx.x & 15) == 0) *jb.dst = jb.dev_norm ? ge_norm_dev(t) : ge_norm_host(t);
            } else if (QL == 4) {
                const ge t = sm_quad(jb.s, jb.P, dtab, pt, pt ? sd.pbits : 0);
                if ((threadIdx.x & 3) == 0) *jb.dst = jb.dev_norm ? ge_norm_dev(t) : ge_norm_host(t);
            } else if (QL == 2) {
                const ge t = sm_pair(jb.s, jb.P, dtab, pt, pt ? sd.pbits : 0);
                if ((threadIdx.x & 1) == 0) *jb.dst = jb.dev_norm ? ge_norm_dev(t) : ge_norm_host(t);
            } else {
                ge t = scalarmult<true>(jb.s, jb.P, &qs[threadIdx.x], dtab, pt, pt ? sd.pbits : 0);
                *jb.dst = jb.dev_norm ? ge_norm_dev(t) : ge_norm_host(t);
            }
        }
    }
}


template <int QL>
void launch_terms_ql(const RegionList& rl, const SlotDev* slots, const ge* G, const ge* H, const ge* g, const ge* h,
                     const ge* dtab, const fe* two_i, hipStream_t s, unsigned lds_pad) {
    const unsigned blocks = (unsigned)((rl.total + TPB - 1) / TPB);
    k_terms<QL><<<blocks, TPB, lds_pad, s>>>(rl, slots, G, H, g, h, dtab, two_i);
}

}  // namespace bp
