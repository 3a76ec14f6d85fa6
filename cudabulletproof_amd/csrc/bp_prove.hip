// bp_prove.hip — gfx950 kernels for the reference's prover:
// generate_range_proof (bulletproof_range_proof.cu:1159-1715), inner_product_prove
// (bulletproof_vectors.cu:277-523) and fix_inner_product_proof (rp.cu:198-235), bit-exact.
//
// A batch of B proofs runs as a short chain of launches; within each launch the work is
// one lane per scalar multiplication (the unit of work, as in the verifier) or one lane per
// sequential chain / per proof:
//   PS_PREP    lane/proof   validate_range_input, aL/aR/sL/sR in tobytes form
//   PS_TERMS0  lane/term    the 4n MSM terms of A and S + g^v, h^gamma, h^alpha, h^rho
//   PS_CHAIN0  lane/chain   point_vector_multi_scalar_mul's sequential accumulation (A11 order)
//   PS_COMMIT  lane/proof   V, A, S; challenges y, z; t0, t1, t2 (sequential inner products)
//   PS_TERMS1  lane/term    g^t1, h^tau1, g^t2, h^tau2
//   PS_TX      lane/proof   T1, T2; x; t, taux, mu; l(x), r(x) (+ the prover's fallback to
//                           l = [t, 0..], r = [1, 0..]); IPA transcript; round-0 scalars
//   per IPA round r: PS_RTERMS (lane/term), PS_RCHAIN (lane/chain), PS_ROUND (lane/proof: L, R,
//                           challenge u, fold of a and b, next round's scalars)
//   PS_FINAL   lane/proof   outputs (+ fix_inner_product_proof); refused values zeroed
// Every order-sensitive fold keeps the reference's order (the arithmetic is not associative).
#include "bp_kernels.h"
#include "ge25519_dev.h"
#include "sha256_dev.h"

#ifndef BP_GTAB
#define BP_GTAB 1
#endif

namespace bp {

namespace {
constexpr int TPB = 256;
__device__ __forceinline__ size_t gid() { return (size_t)blockIdx.x * blockDim.x + threadIdx.x; }
inline unsigned nblk(size_t items) { return (unsigned)((items + TPB - 1) / TPB); }
}  // namespace

// Base b's prefix-table row (ProveWs::ptab), or null without tables.
__device__ __forceinline__ const ge* prow(const ProveWs& ws, int b) {
    return ws.ptab ? ws.ptab + ((size_t)b << ws.pbits) : nullptr;
}

// ge25519_normalize(scalarmult(tobytes(s), P)) — the scalar is already in tobytes form.
__device__ __forceinline__ ge sm_norm(const fe& s, const ge& P, geq* qslot, const ge* __restrict__ dtab,
                                      const ge* pt, int K) {
    return ge_norm_host(scalarmult<true>(s, P, qslot, dtab, pt, pt ? K : 0));
}

// sequential inner product, field_vector_inner_product (vectors.cu:101-114)
__device__ __forceinline__ fe ip_seq(const fe* a, const fe* b, int n) {
    fe acc = fe_set(0);
    for (int i = 0; i < n; i++) acc = fe_add(acc, fe_mul(a[i], b[i]));
    return acc;
}

// validate_range_input (rp.cu:238-264) on the tobytes form of v (n < 256).
__device__ __forceinline__ bool validate_range(const fe& vc, int n) {
    int bi = n >> 3, bit = n & 7;
    if ((fe_byte(vc, bi) >> bit) & 1) return false;
    for (int i = bi + (bit == 7 ? 1 : 0); i < 32; i++)
        if (fe_byte(vc, i)) return false;
    return true;
}

__device__ __forceinline__ fe bit_fe(const fe& vc, int i) { return fe_set((vc.v[i >> 6] >> (i & 63)) & 1); }

// Work lists.  A zero scalar's term is a constant (ge25519_scalarmult leaves the identity
// doubled 256 times whatever the point: dtab[256], normalized dtab[257]), so those items are
// written directly; the rest are queued by cost class — light (<= 64 significant bits: the
// aL bits, the value) and heavy — so that a wave does not run a 255-bit scalar-mult for one
// lane while 63 others idle.  One lane per proof reserves its items with one atomic per class.
__device__ __forceinline__ int sclass(const fe& s) {
    if (s.v[3] | s.v[2] | s.v[1]) return 2;
    return s.v[0] ? 1 : 0;
}

// class_of(k): 0 constant (written by the caller), 1 light, 2 heavy, 3 from the per-batch table
template <typename ClassOf>
__device__ __forceinline__ void queue_items(const ProveWs& ws, size_t p, int per, ClassOf class_of) {
    unsigned nh = 0, nl = 0;
    for (int k = 0; k < per; k++) {
        int c = class_of(k);
        nh += c == 2;
        nl += c == 1;
    }
    unsigned bh = nh ? atomicAdd(&ws.cnt[0], nh) : 0, bl = nl ? atomicAdd(&ws.cnt[1], nl) : 0;
    for (int k = 0; k < per; k++) {
        int c = class_of(k);
        uint32_t id = (uint32_t)(p * per + k);
        if (c == 2) ws.list[bh++] = id;
        else if (c == 1) ws.list[ws.cap + bl++] = id;
    }
}

// The i-th queued item of a list-driven launch (heavy first), or false past the end.
__device__ __forceinline__ bool next_item(const ProveWs& ws, size_t i, uint32_t& id) {
    const unsigned ch = ws.cnt[0], cl = ws.cnt[1];
    if (i < ch) { id = ws.list[i]; return true; }
    if (i < (size_t)ch + cl) { id = ws.list[ws.cap + (i - ch)]; return true; }
    return false;
}

// terms0 item k's scalar (tobytes form, or the raw alpha / rho bytes)
__device__ __forceinline__ fe terms0_scalar(const ProveIn& in, const ProveWs& ws, size_t p, int k) {
    const int n = in.n;
    if (k < 4 * n) return ws.ps[p * 4 * n + k];
    k -= 4 * n;
    if (k == 0) return fe_canon(in.v[p]);
    if (k == 1) return fe_canon(in.gamma[p]);
    return in.rnd[p * 4 + (k - 2)];
}

// ---------------------------------------------------------------- PS_PREP
__global__ __launch_bounds__(TPB) void k_prove_prep(ProveIn in, ProveWs ws, const ge* __restrict__ dtab) {
    size_t p = gid();
    if (p >= (size_t)in.B) return;
    const int n = in.n;
    fe vc = fe_canon(in.v[p]);
    ws.valid[p] = validate_range(vc, n) ? 1 : 0;
    const fe one = fe_set(1);
    fe* ps = ws.ps + p * 4 * n;
    for (int i = 0; i < n; i++) {                      // rp.cu:1218-1238, 1246-1252
        fe aL = bit_fe(vc, i);
        ps[i] = aL;
        ps[n + i] = fe_canon(fe_sub(aL, one));
        ps[2 * n + i] = fe_canon(in.sL[p * n + i]);
        ps[3 * n + i] = fe_canon(in.sR[p * n + i]);
    }
    const int per = 4 * n + 4;
    ge* pt = ws.pterm + p * per;
    for (int k = 0; k < per; k++)   // zero scalars: the constant term (raw for h^alpha, h^rho)
        if (sclass(terms0_scalar(in, ws, p, k)) == 0) pt[k] = dtab[k < 4 * n + 2 ? 257 : 256];
    // aR_i = sub(0, 1) wherever aL_i = 0, and aL_i = 1 otherwise: the same scalar on the same
    // generator in every proof, so those terms are ws.ctab[i] (aR H_i) and ws.ctab[n + i] (1 G_i),
    // computed once per batch by the first 2n lanes of k_prove_terms0
    queue_items(ws, p, per, [&](int k) {
        if (BP_GTAB && k < n && ps[k].v[0]) return 3;
        if (k >= n && k < 2 * n && !(ps[k - n].v[0])) return 3;
        return sclass(terms0_scalar(in, ws, p, k));
    });
}

// ---------------------------------------------------------------- terms0 lane sort
// The heavy items are random 255-bit scalars (sL, sR, gamma): a wave runs as long as its
// longest chain, so the heavy list is counting-sorted by chain length (sm_ops) into slist,
// longest first (the same scheme as the MSM's k_ops_*).
// 256-thread blocks: a 1024-thread block needs a whole CU's wave slots and waits behind the other
// stream's running terms0 (in the r03q trace the scatter took 28 ms per launch that way)
constexpr int SORT_T = 256;
__global__ __launch_bounds__(TPB) void k_prove_sort_hist(ProveIn in, ProveWs ws) {
    __shared__ unsigned hb[MSM_BINS];
    for (int k = threadIdx.x; k < MSM_BINS; k += TPB) hb[k] = 0;
    __syncthreads();
    const size_t i = gid(), per = 4 * (size_t)in.n + 4;
    if (i < ws.cnt[0]) {
        const uint32_t id = ws.list[i];
        atomicAdd(&hb[sm_ops_prefix(terms0_scalar(in, ws, id / per, (int)(id % per)), ws.ptab ? ws.pbits : 0)], 1u);
    }
    __syncthreads();
    for (int k = threadIdx.x; k < MSM_BINS; k += TPB)
        if (hb[k]) atomicAdd(&ws.sbins[k], hb[k]);
}

__global__ __launch_bounds__(SORT_T) void k_prove_sort_scatter(ProveIn in, ProveWs ws) {
    __shared__ unsigned cnt[MSM_BINS], base[MSM_BINS];
    for (int k = threadIdx.x; k < MSM_BINS; k += SORT_T) cnt[k] = 0;
    __syncthreads();
    const size_t i = (size_t)blockIdx.x * SORT_T + threadIdx.x, per = 4 * (size_t)in.n + 4;
    int key = 0;
    unsigned rank = 0;
    uint32_t id = 0;
    const bool live = i < ws.cnt[0];
    if (live) {
        id = ws.list[i];
        key = sm_ops_prefix(terms0_scalar(in, ws, id / per, (int)(id % per)), ws.ptab ? ws.pbits : 0);
        rank = atomicAdd(&cnt[key], 1u);
    }
    __syncthreads();
    for (int k = threadIdx.x; k < MSM_BINS; k += SORT_T)
        if (cnt[k]) base[k] = atomicAdd(&ws.sbins[k], cnt[k]);
    __syncthreads();
    if (live) ws.slist[base[key] + rank] = id;
}

// ---------------------------------------------------------------- PS_TERMS0
// item k of proof p (4n+4 items): k < 4n the MSM term ps[k] * (G|H)[k % n], host-normalized
// (vectors.cu:204-206); then g^v, h^gamma (pedersen_commit, rp.cu:277-297: normalized) and the
// raw h^alpha, h^rho of rp.cu:1268, :1280 (not normalized).
__global__ __launch_bounds__(TPB, 3) void k_prove_terms0(ProveIn in, ProveWs ws, const ge* __restrict__ G,
                                                      const ge* __restrict__ H, const ge* __restrict__ g,
                                                      const ge* __restrict__ h, const ge* __restrict__ dtab) {
    __shared__ geq qs[TPB];
    const int n = in.n;
    const size_t per = 4 * (size_t)n + 4;
    // lanes [0, 2n): the table ws.ctab[j] = N(sm(tobytes(sub(0, 1)), H_j)) (the aR_j term of every
    // proof with aL_j = 0), ws.ctab[n + j] = N(sm(1, G_j)) (the aL_j term where aL_j = 1); then the
    // queued items
    const size_t i = gid();
    uint32_t id = 0;
    if (i >= 2 * (size_t)n) {
        const size_t q = i - 2 * n;
        if (ws.slist && q < ws.cnt[0]) id = ws.slist[q];
        else if (!next_item(ws, q, id)) return;
    }
    size_t p = id / per;
    int k = (int)(id % per);
    // operands are selected per lane and ONE scalar-mult follows: two call sites in one wave
    // would run both loops back to back (divergence), ~1.6x the instructions
    fe s;
    ge P;
    bool norm = true;
    int base;                                       // prefix-table row of P
    ge* dst = ws.pterm + id;
    if (i < 2 * (size_t)n) {
        const bool hs = i < (size_t)n;
        P = hs ? H[i] : G[i - n];
        base = hs ? n + (int)i : (int)i - n;
        s = hs ? fe_canon(fe_sub(fe_set(0), fe_set(1))) : fe_set(1);   // k_prove_prep's aR (aL = 0), aL = 1
        dst = ws.ctab + i;
    } else if (k < 4 * n) {
        int blk = k / n, j = k % n;
        P = (blk & 1) ? H[j] : G[j];
        base = (blk & 1) ? n + j : j;
        s = ws.ps[p * 4 * n + k];
    } else {
        k -= 4 * n;
        P = k == 0 ? *g : *h;
        base = k == 0 ? 2 * n + 1 : 2 * n;
        s = terms0_scalar(in, ws, p, 4 * n + k);
        norm = k < 2;                               // alpha_bytes / rho_bytes: raw, not normalized
    }
    const ge* pt = prow(ws, base);
    ge r = scalarmult<true>(s, P, &qs[threadIdx.x], dtab, pt, pt ? ws.pbits : 0);
    *dst = norm ? ge_norm_host(r) : r;
}

// ---------------------------------------------------------------- chains
// point_vector_multi_scalar_mul's accumulation (vectors.cu:208-223): acc = t_0, then
// acc = N(acc + t_i), final N.  Chain j of proof p: count terms at base + p*pps + j*pcs.
__global__ __launch_bounds__(TPB) void k_prove_chain(const ge* __restrict__ terms, size_t pps, size_t pcs, int count,
                                                     int per_proof, ge* out, int B) {
    size_t c = gid();
    if (c >= (size_t)B * per_proof) return;
    size_t p = c / per_proof;
    int j = (int)(c % per_proof);
    const ge* t = terms + p * pps + (size_t)j * pcs;
    ge acc = t[0];
    for (int i = 1; i < count; i++) acc = ge_norm_host(ge_add(acc, t[i]));
    out[c] = ge_norm_host(acc);
}

// chain set 0 (aL G | aR H | sL G | sR H): as k_prove_chain, the table terms from ws.ctab
__global__ __launch_bounds__(TPB) void k_prove_chain0(ProveIn in, ProveWs ws) {
    size_t c = gid();
    if (c >= (size_t)in.B * 4) return;
    const int n = in.n;
    size_t p = c / 4;
    int j = (int)(c % 4);
    const ge* t = ws.pterm + p * (4 * (size_t)n + 4) + (size_t)j * n;
    const fe* aL = ws.ps + p * 4 * (size_t)n;
    auto term = [&](int i) {
        if (BP_GTAB && j == 0 && aL[i].v[0]) return ws.ctab[n + i];
        return (j == 1 && !aL[i].v[0]) ? ws.ctab[i] : t[i];
    };
    ge acc = term(0);
    for (int i = 1; i < n; i++) acc = ge_norm_host(ge_add(acc, term(i)));
    ws.chain[c] = ge_norm_host(acc);
}

// ---------------------------------------------------------------- PS_COMMIT
__global__ __launch_bounds__(TPB) void k_prove_commit(ProveIn in, ProveWs ws, const fe* __restrict__ two_i) {
    size_t p = gid();
    if (p >= (size_t)in.B) return;
    const int n = in.n;
    const ge* pt = ws.pterm + p * (4 * (size_t)n + 4) + 4 * n;
    const ge* ch = ws.chain + p * 4;
    ge V = ge_norm_host(ge_add(pt[0], pt[1]));                     // pedersen_commit (rp.cu:293-296)
    ge A = ge_norm_host(ge_add(ge_add(pt[2], ch[0]), ch[1]));      // rp.cu:1272-1274
    ge S = ge_norm_host(ge_add(ge_add(pt[3], ch[2]), ch[3]));      // rp.cu:1284-1286
    ws.pts[p * 5 + 0] = V;
    ws.pts[p * 5 + 1] = A;
    ws.pts[p * 5 + 2] = S;
    fe y = chal_y(V, A, S);                                         // challenge.cu:24-58
    fe z = chal_z(y);
    fe z2 = fe_mul(z, z);
    // t0 = <aL - z, y^n o (aR + z)> + z^2 <1^n, 2^n>, t1 = <sL, y^n o (aR + z)> + <aL - z, y^n o sR>,
    // t2 = <sL, y^n o sR>   (rp.cu:1358-1430): four sequential folds in index order, one pass.
    fe vc = fe_canon(in.v[p]);
    const fe one = fe_set(1);
    fe py = one, a0 = fe_set(0), a1 = fe_set(0), a2 = fe_set(0), a3 = fe_set(0), s2 = fe_set(0);
    for (int i = 0; i < n; i++) {
        if (i > 0) py = fe_mul(py, y);                             // powers_of (rp.cu:299-313)
        fe aL = bit_fe(vc, i), aR = fe_sub(aL, one);
        fe lz = fe_sub(aL, z);
        fe u1 = fe_mul(py, fe_add(aR, z));
        fe u2 = fe_mul(py, in.sR[p * n + i]);
        fe sL = in.sL[p * n + i];
        a0 = fe_add(a0, fe_mul(lz, u1));
        a1 = fe_add(a1, fe_mul(sL, u1));
        a2 = fe_add(a2, fe_mul(lz, u2));
        a3 = fe_add(a3, fe_mul(sL, u2));
        s2 = fe_add(s2, two_i[i]);                                 // <1^n, 2^n> (rp.cu:1396-1398)
    }
    fe t0 = fe_add(a0, fe_mul(z2, s2));
    fe t1 = fe_add(a1, a2);
    fe* st = ws.st + p * 8;
    st[0] = y; st[1] = z; st[2] = z2; st[3] = t0; st[4] = t1; st[5] = a3;
    fe* ts = ws.tsc + p * 4;
    ts[0] = fe_canon(t1);
    ts[1] = fe_canon(in.rnd[p * 4 + 2]);
    ts[2] = fe_canon(a3);
    ts[3] = fe_canon(in.rnd[p * 4 + 3]);
}

// ---------------------------------------------------------------- PS_TERMS1: T1 = g^t1 h^tau1, T2 = g^t2 h^tau2
__global__ __launch_bounds__(TPB, 3) void k_prove_terms1(ProveIn in, ProveWs ws, const ge* __restrict__ g,
                                                      const ge* __restrict__ h, const ge* __restrict__ dtab) {
    __shared__ geq qs[TPB];
    size_t i = gid();
    if (i >= (size_t)in.B * 4) return;
    ws.tt[i] = sm_norm(ws.tsc[i], (i & 1) ? *h : *g, &qs[threadIdx.x], dtab, prow(ws, 2 * in.n + ((i & 1) ? 0 : 1)),
                       ws.pbits);
}

// round-r scalars (inner_product_prove, vectors.cu:345-376): c_L = <a_L, b_R>, c_R = <a_R, b_L> and the
// four MSMs' scalars in tobytes form: a_L | b_R | a_R | b_L.
__device__ __forceinline__ void round_prep(const ProveWs& ws, size_t p, int n, int np, const ge* __restrict__ dtab) {
    const fe* a = ws.acur + p * n;
    const fe* b = ws.bcur + p * n;
    fe* cs = ws.csc + p * 2;
    cs[0] = fe_canon(ip_seq(a, b + np, np));
    cs[1] = fe_canon(ip_seq(a + np, b, np));
    fe* sc = ws.iscal + p * 2 * n;
    for (int j = 0; j < np; j++) {
        sc[j] = fe_canon(a[j]);
        sc[np + j] = fe_canon(b[np + j]);
        sc[2 * np + j] = fe_canon(a[np + j]);
        sc[3 * np + j] = fe_canon(b[j]);
    }
    const int per = 4 * np + 2;
    auto scalar_of = [&](int k) { return k < 4 * np ? sc[k] : cs[k - 4 * np]; };
    ge* it = ws.iterm + p * (2 * (size_t)n + 2);
    for (int k = 0; k < per; k++)   // zero scalars: the constant term (raw for c_L Q, c_R Q)
        if (sclass(scalar_of(k)) == 0) it[k] = dtab[k < 4 * np ? 257 : 256];
    queue_items(ws, p, per, [&](int k) { return sclass(scalar_of(k)); });
}

// ---------------------------------------------------------------- PS_TX
__global__ __launch_bounds__(TPB) void k_prove_tx(ProveIn in, ProveWs ws, const fe* __restrict__ two_i,
                                                  const ge* __restrict__ dtab) {
    size_t p = gid();
    if (p >= (size_t)in.B) return;
    const int n = in.n;
    const ge* tt = ws.tt + p * 4;
    ge T1 = ge_norm_host(ge_norm_host(ge_add(tt[0], tt[1])));     // pedersen_commit + rp.cu:1444
    ge T2 = ge_norm_host(ge_norm_host(ge_add(tt[2], tt[3])));
    ws.pts[p * 5 + 3] = T1;
    ws.pts[p * 5 + 4] = T2;
    fe x = chal_x(T1, T2);                                          // challenge.cu:61-77
    fe x2 = fe_mul(x, x);
    fe* st = ws.st + p * 8;
    const fe y = st[0], z = st[1], z2 = st[2];
    fe t = fe_add(fe_add(st[3], fe_mul(st[4], x)), fe_mul(st[5], x2));   // rp.cu:1470-1480
    const fe* rnd = in.rnd + p * 4;
    fe taux = fe_add(fe_mul(rnd[2], x), fe_mul(rnd[3], x2));            // rp.cu:1487-1490
    fe mu = fe_add(rnd[0], fe_mul(rnd[1], x));                          // rp.cu:1497-1499
    // l(x) = aL - z + sL x, r(x) = y^n o (aR + z + sR x) + z^2 2^n  (rp.cu:1515-1580)
    fe vc = fe_canon(in.v[p]);
    const fe one = fe_set(1);
    fe* a = ws.acur + p * n;
    fe* b = ws.bcur + p * n;
    fe py = one, ip = fe_set(0);
    for (int i = 0; i < n; i++) {
        if (i > 0) py = fe_mul(py, y);
        fe aL = bit_fe(vc, i), aR = fe_sub(aL, one);
        fe l = fe_add(fe_sub(aL, z), fe_mul(in.sL[p * n + i], x));
        fe r = fe_add(fe_mul(fe_add(fe_add(aR, z), fe_mul(in.sR[p * n + i], x)), py), fe_mul(z2, two_i[i]));
        a[i] = l;
        b[i] = r;
        ip = fe_add(ip, fe_mul(l, r));
    }
    if (!fe_eq(fe_canon(ip), fe_canon(t))) {                         // rp.cu:1604-1622
        for (int i = 0; i < n; i++) {
            a[i] = fe_set(0);
            b[i] = fe_set(0);
        }
        a[0] = t;
        b[0] = one;
    }
    st[6] = t;
    st[7] = chal_ip_start(t, taux, mu);                             // the IPA transcript (rp.cu:1636-1650)
    fe* m = ws.misc + p * 4;
    m[0] = taux;
    m[1] = mu;
    m[2] = fe_set(0);                                               // x (ip_proof.x) until round 0
    if (in.L > 0) round_prep(ws, p, n, n >> 1, dtab);
}

// ---------------------------------------------------------------- IPA round r
// item k of proof p (4n'+2 items): a_L_j G[n'+j] | b_R_j H[j] | a_R_j G[j] | b_L_j H[n'+j] (host-normalized
// MSM terms, vectors.cu:397-398, :430-431) | c_L Q | c_R Q (raw, :402-404, :435-437).  G, H are the
// ORIGINAL generators every round (the prover never folds them).
__global__ __launch_bounds__(TPB, 3) void k_prove_rterms(ProveIn in, ProveWs ws, int np, const ge* __restrict__ G,
                                                      const ge* __restrict__ H, const ge* __restrict__ Q,
                                                      const ge* __restrict__ dtab) {
    __shared__ geq qs[TPB];
    const int n = in.n;
    const size_t per = 4 * (size_t)np + 2;
    uint32_t id;
    // grid-stride over the queued items: the lists hold ~2 non-zero items per proof when the prover
    // takes its l = [t, 0..], r = [1, 0..] fallback, so a grid of B (4n' + 2) lanes would be almost
    // all empty waves, and under another stream's running terms0 every one of them waits for a slot
    for (size_t i = gid(); next_item(ws, i, id); i += (size_t)gridDim.x * TPB) {
        size_t p = id / per;
        int k = (int)(id % per);
        fe s;
        ge P;
        int base;
        const bool msm = k < 4 * np;
        if (msm) {
            int blk = k / np, j = k % np;
            P = blk == 0 ? G[np + j] : blk == 1 ? H[j] : blk == 2 ? G[j] : H[np + j];
            base = blk == 0 ? np + j : blk == 1 ? n + j : blk == 2 ? j : n + np + j;
            s = ws.iscal[p * 2 * n + k];
        } else {
            P = *Q;
            base = 2 * n;   // Q = h
            s = ws.csc[p * 2 + (k - 4 * np)];
        }
        const ge* pt = prow(ws, base);
        ge r = scalarmult<true>(s, P, &qs[threadIdx.x], dtab, pt, pt ? ws.pbits : 0);   // one call site (k_prove_terms0)
        ws.iterm[p * (2 * (size_t)n + 2) + k] = msm ? ge_norm_host(r) : r;
    }
}

__global__ __launch_bounds__(TPB) void k_prove_round(ProveIn in, ProveWs ws, ProveOut out, int r,
                                                     const ge* __restrict__ dtab) {
    size_t p = gid();
    if (p >= (size_t)in.B) return;
    const int n = in.n, np = n >> (r + 1);
    const ge* ch = ws.chain + p * 4;
    const ge* tq = ws.iterm + p * (2 * (size_t)n + 2) + 4 * np;
    ge L = ge_norm_host(ge_add(ge_add(ge_add(ge_zero(), ch[0]), ch[1]), tq[0]));   // vectors.cu:407-411
    ge R = ge_norm_host(ge_add(ge_add(ge_add(ge_zero(), ch[2]), ch[3]), tq[1]));   // :440-444
    out.L[p * in.L + r] = L;
    out.R[p * in.L + r] = R;
    fe* st = ws.st + p * 8;
    fe u = chal_ip(st[7], L.X, R.X);                                // vectors.cu:450-466
    st[7] = u;
    if (r == 0) ws.misc[p * 4 + 2] = u;                              // proof->x (vectors.cu:472-474)
    fe ui = fe_invert(u);
    fe* a = ws.acur + p * n;
    fe* b = ws.bcur + p * n;
    for (int j = 0; j < np; j++) {                                  // vectors.cu:489-499
        fe na = fe_add(fe_mul(ui, a[j]), fe_mul(u, a[np + j]));
        fe nb = fe_add(fe_mul(u, b[j]), fe_mul(ui, b[np + j]));
        a[j] = na;
        b[j] = nb;
    }
    if (r + 1 < in.L) round_prep(ws, p, n, np >> 1, dtab);
}

// ---------------------------------------------------------------- PS_FINAL (+ fix_inner_product_proof)
__global__ __launch_bounds__(TPB) void k_prove_final(ProveIn in, ProveWs ws, ProveOut out) {
    size_t p = gid();
    if (p >= (size_t)in.B) return;
    const bool ok = ws.valid[p] != 0;
    out.valid[p] = ok ? 1 : 0;
    const ge* pts = ws.pts + p * 5;
    const ge O = ge_zero();
    const fe Z = fe_set(0);
    // a refused value leaves V, A, S, T1, T2 = identity and taux, mu, t = 0 (rp.cu:1176-1188)
    out.V[p] = ok ? pts[0] : O;
    out.A[p] = ok ? pts[1] : O;
    out.S[p] = ok ? pts[2] : O;
    out.T1[p] = ok ? pts[3] : O;
    out.T2[p] = ok ? pts[4] : O;
    const fe t = ws.st[p * 8 + 6];
    const fe* m = ws.misc + p * 4;
    out.taux[p] = ok ? m[0] : Z;
    out.mu[p] = ok ? m[1] : Z;
    out.t[p] = ok ? t : Z;
    out.c[p] = ok ? t : Z;
    out.x[p] = ok ? m[2] : Z;
    out.a[p] = ok ? t : Z;
    out.b[p] = ok ? fe_set(1) : Z;
    if (!ok) {
        const ge zero{Z, Z, Z, Z};
        for (int r = 0; r < in.L; r++) {
            out.L[p * in.L + r] = zero;
            out.R[p * in.L + r] = zero;
        }
    }
}

void launch_prove(int stage, int r, const ProveIn& in, const ProveWs& ws, const ProveOut& out, const ge* G,
                  const ge* H, const ge* g, const ge* h, const ge* dtab, const fe* two_i, hipStream_t s) {
    const size_t B = in.B;
    const int n = in.n;
    switch (stage) {
        case PS_PREP:
            (void)hipMemsetAsync(ws.cnt, 0, 2 * sizeof(unsigned), s);
            k_prove_prep<<<nblk(B), TPB, 0, s>>>(in, ws, dtab);
            break;
        case PS_SORT0:
            if (ws.slist) {   // heavy list -> chain-length order (the list length is on the device)
                const size_t cap = ws.cap;
                (void)hipMemsetAsync(ws.sbins, 0, MSM_BINS * sizeof(unsigned), s);
                k_prove_sort_hist<<<nblk(cap), TPB, 0, s>>>(in, ws);
                launch_ops_scan(ws.sbins, 1, s);
                k_prove_sort_scatter<<<(unsigned)((cap + SORT_T - 1) / SORT_T), SORT_T, 0, s>>>(in, ws);
            }
            break;
        case PS_TERMS0: {
            // the lists hold at most 2n + 4 items per proof (sL, sR, v, gamma, alpha, rho): every aL / aR
            // term is a zero-scalar constant or a ctab entry (BP_GTAB), so the grid stops there
            const size_t per_max = BP_GTAB ? 2 * (size_t)n + 4 : 4 * (size_t)n + 4;
            k_prove_terms0<<<nblk(B * per_max + 2 * n), TPB, 0, s>>>(in, ws, G, H, g, h, dtab);
            break;
        }
        case PS_CHAIN0: k_prove_chain0<<<nblk(B * 4), TPB, 0, s>>>(in, ws); break;
        case PS_COMMIT: k_prove_commit<<<nblk(B), TPB, 0, s>>>(in, ws, two_i); break;
        case PS_TERMS1: k_prove_terms1<<<nblk(B * 4), TPB, 0, s>>>(in, ws, g, h, dtab); break;
        case PS_TX:
            (void)hipMemsetAsync(ws.cnt, 0, 2 * sizeof(unsigned), s);
            k_prove_tx<<<nblk(B), TPB, 0, s>>>(in, ws, two_i, dtab);
            break;
        case PS_RTERMS: {
            int np = n >> (r + 1);
            // at most RTERMS_BLOCKS blocks (4 waves per SIMD over the GPU), grid-stride over the items
            constexpr unsigned RTERMS_BLOCKS = 1024;
            const unsigned nb = nblk(B * (4 * (size_t)np + 2));
            k_prove_rterms<<<nb < RTERMS_BLOCKS ? nb : RTERMS_BLOCKS, TPB, 0, s>>>(in, ws, np, G, H, h, dtab);
            break;
        }
        case PS_RCHAIN: {
            int np = n >> (r + 1);
            k_prove_chain<<<nblk(B * 4), TPB, 0, s>>>(ws.iterm, 2 * (size_t)n + 2, np, np, 4, ws.chain, in.B);
            break;
        }
        case PS_ROUND:
            (void)hipMemsetAsync(ws.cnt, 0, 2 * sizeof(unsigned), s);
            k_prove_round<<<nblk(B), TPB, 0, s>>>(in, ws, out, r, dtab);
            break;
        case PS_FINAL: k_prove_final<<<nblk(B), TPB, 0, s>>>(in, ws, out); break;
    }
}

}  // namespace bp
