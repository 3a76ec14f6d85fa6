// bp_kernels.hip — gfx950 kernels for the MSM / inner-product-argument verify path.
//
// One lane computes one scalar multiplication (the unit of work); waves
// whose lanes share a scalar take the scalar-branch loop, others the per-lane loop
// (ge25519_dev.h). Reductions follow the reference's canonical pairwise tree order
// (cuda_bulletproof_kernels.cu:162-168) through LDS; every order-sensitive fold keeps
// the reference's order, because the arithmetic is not associative.
#include "bp_kernels.h"
#include "ge25519_dev.h"
#include "ge25519_quad.h"
#include "sha256_dev.h"

namespace bp {

constexpr int TPB = 256;   // threads per block for lane-per-item kernels
#ifndef BP_TERMS_OCC
#define BP_TERMS_OCC 4   // k_terms blocks per CU the register budget is sized for
#endif


__device__ __forceinline__ size_t gid() { return (size_t)blockIdx.x * blockDim.x + threadIdx.x; }

// ------------------------------------------------------------------ tables
// dtab[k] = k successive ge25519_add(r, r) of the identity (0,1,1,0): the state of
// ge25519_scalarmult after k leading zero bits (curve25519_ops.cu:399-414); dtab[257] =
// ge25519_normalize(dtab[256]), the normalized result of any point times the zero scalar.
// two_i[i] = i successive fe25519_mul(., 2) from 1 (bulletproof_range_proof.cu:705-712).
__global__ void k_init_tables(ge* dtab, fe* two_i, int nmax) {
    if (gid() != 0) return;
    ge r = ge_zero();
    dtab[0] = r;
    for (int k = 1; k <= 256; k++) {
        r = ge_dbl(r);
        dtab[k] = r;
    }
    dtab[257] = ge_norm_host(r);   // a zero scalar's host-normalized term, whatever the point
    fe two = fe_add(fe_set(1), fe_set(1));
    fe t = fe_set(1);
    for (int i = 0; i < nmax; i++) {
        two_i[i] = t;
        t = fe_mul(t, two);
    }
}

void launch_init_tables(ge* dtab, fe* two_i, int nmax, hipStream_t s) {
    k_init_tables<<<1, 64, 0, s>>>(dtab, two_i, nmax);
}

// tab[b << K | p] = the first K steps of ge25519_scalarmult (curve25519_ops.cu:397-415) on base b
// for a scalar whose top K bits are p, from the identity: one add(r, r) per bit and one add(r, P)
// per set bit — the per-lane step of sm_lane_loop, so the same operations as the verify kernels.
__global__ __launch_bounds__(TPB) void k_prefix_tables(ge* tab, const ge* __restrict__ G, const ge* __restrict__ H,
                                                       const ge* __restrict__ h, const ge* __restrict__ g, int n,
                                                       int K, size_t total) {
    const size_t i = gid();
    if (i >= total) return;
    const size_t b = i >> K;
    const uint32_t p = (uint32_t)(i & ((1ull << K) - 1));
    const ge* P = b < (size_t)n ? &G[b] : b < 2 * (size_t)n ? &H[b - n] : b == 2 * (size_t)n ? h : g;
    if (!P) return;
    const geq q = ge_prep(*P);
    ge r = ge_zero();
    for (int j = K - 1; j >= 0; j--) {
        r = ge_add_sel<false>(r, &q, false);
        if ((p >> j) & 1) r = ge_add_sel<false>(r, &q, true);
    }
    tab[i] = r;
}

void launch_prefix_tables(ge* tab, const ge* G, const ge* H, const ge* h, const ge* g, int n, int K, hipStream_t s) {
    const size_t total = (size_t)(2 * n + 2) << K;
    k_prefix_tables<<<(unsigned)((total + TPB - 1) / TPB), TPB, 0, s>>>(tab, G, H, h, g, n, K, total);
}

// ------------------------------------------------------------------ MSM
// pts[seg*m + i] = Ndev(scalarmult(rawbytes(scal[seg*m+i]), P[i])) — point_scalar_mul_kernel
// (cuda_bulletproof_kernels.cu:26-42); the scalar bytes are the raw limbs (device tobytes).
// `perm` (nullable) maps lane -> item: the lanes of a wave take items of equal length, so no
// lane idles while the longest scalar of its wave finishes (below).
// `pm`: the point of item i is P[i % pm] (a batch of MSMs over the same points; pm = total for one).
#ifndef BP_MSM_TPB
#define BP_MSM_TPB 256   // k_msm_points block size
#endif
constexpr int MSM_TPB = BP_MSM_TPB;
// `ptab` / K (nullable / 0): prefix tables of the points as bases (point b's rows at b << K),
// when the points are generators with tables (hipbp_msm_batch_gens).
__global__ __launch_bounds__(MSM_TPB, 768 / MSM_TPB) void k_msm_points(ge* pts, const fe* __restrict__ scal,
                                                    const ge* __restrict__ P, size_t total, size_t pm,
                                                    const uint32_t* __restrict__ perm,
                                                    const ge* __restrict__ dtab, const ge* __restrict__ ptab,
                                                    int K) {
    __shared__ geq qs[MSM_TPB];
    size_t i = gid();
    if (i >= total) return;
    if (perm) i = perm[i];
    const size_t b = pm == total ? i : i % pm;
    ge r = scalarmult<true>(scal[i], P[b], &qs[threadIdx.x], dtab, ptab ? ptab + (b << K) : nullptr, ptab ? K : 0);
    pts[i] = ge_norm_dev(r);
}

constexpr int OPS_BINS = MSM_BINS;

__global__ void k_ops_zero(unsigned* bins) {
    for (int k = threadIdx.x; k < OPS_BINS; k += blockDim.x) bins[k] = 0;
}

__global__ __launch_bounds__(TPB) void k_ops_hist(unsigned* bins, const fe* __restrict__ scal, size_t n, int K) {
    __shared__ unsigned h[OPS_BINS];
    for (int k = threadIdx.x; k < OPS_BINS; k += TPB) h[k] = 0;
    __syncthreads();
    size_t i = gid();
    if (i < n) atomicAdd(&h[sm_ops_prefix(scal[i], K)], 1u);
    __syncthreads();
    for (int k = threadIdx.x; k < OPS_BINS; k += TPB)
        if (h[k]) atomicAdd(&bins[k], h[k]);
}

// bins -> start offsets (exclusive scan in one block), longest first when asked (the longest
// waves are then dispatched first and the kernel's tail is made of the shortest ones).
constexpr int SCAN_T = 1024;
static_assert(OPS_BINS <= SCAN_T, "one scan block");
__global__ __launch_bounds__(SCAN_T) void k_ops_scan(unsigned* bins, int longest_first) {
    __shared__ unsigned a[SCAN_T];
    const int t = threadIdx.x;
    const int k = longest_first ? OPS_BINS - 1 - t : t;
    const unsigned v = t < OPS_BINS ? bins[k] : 0u;
    a[t] = v;
    __syncthreads();
    for (int off = 1; off < SCAN_T; off <<= 1) {   // Hillis-Steele inclusive scan
        unsigned x = t >= off ? a[t - off] : 0u;
        __syncthreads();
        a[t] += x;
        __syncthreads();
    }
    if (t < OPS_BINS) bins[k] = a[t] - v;
}

// Block-aggregated scatter: ranks within the block from LDS atomics, one global atomic per
// (block, bin) to reserve the block's range (per-item global atomics on ~100 hot bins
// serialise: 1.7 ms for 2^20 items).
__global__ __launch_bounds__(SCAN_T) void k_ops_scatter(uint32_t* perm, unsigned* offs, const fe* __restrict__ scal,
                                                        size_t n, int K) {
    __shared__ unsigned cnt[OPS_BINS], base[OPS_BINS];
    for (int k = threadIdx.x; k < OPS_BINS; k += SCAN_T) cnt[k] = 0;
    __syncthreads();
    size_t i = (size_t)blockIdx.x * SCAN_T + threadIdx.x;
    int key = 0;
    unsigned rank = 0;
    if (i < n) {
        key = sm_ops_prefix(scal[i], K);
        rank = atomicAdd(&cnt[key], 1u);
    }
    __syncthreads();
    for (int k = threadIdx.x; k < OPS_BINS; k += SCAN_T)
        if (cnt[k]) base[k] = atomicAdd(&offs[k], cnt[k]);
    __syncthreads();
    if (i < n) perm[base[key] + rank] = (uint32_t)i;
}

void launch_ops_scan(unsigned* bins, int longest_first, hipStream_t s) {
    k_ops_scan<<<1, SCAN_T, 0, s>>>(bins, longest_first);
}

void launch_msm_points(ge* pts, const fe* scal, const ge* P, size_t m, uint32_t* perm, unsigned* bins,
                       const ge* dtab, hipStream_t s, size_t pm, const ge* ptab, int K) {
    if (!ptab) K = 0;
    if (!pm) pm = m;
    size_t blocks = (m + TPB - 1) / TPB;
    static const int sort_mode = getenv("HIPBP_MSM_SORT") ? atoi(getenv("HIPBP_MSM_SORT")) : 1;
    if (!sort_mode) perm = nullptr;
    if (perm && bins && m >= MSM_SORT_MIN && m <= 0xFFFFFFFFull) {   // a counting sort of the items by chain length
        k_ops_zero<<<1, 64, 0, s>>>(bins);
        k_ops_hist<<<blocks, TPB, 0, s>>>(bins, scal, m, K);
        k_ops_scan<<<1, SCAN_T, 0, s>>>(bins, sort_mode == 1);
        k_ops_scatter<<<(unsigned)((m + SCAN_T - 1) / SCAN_T), SCAN_T, 0, s>>>(perm, bins, scal, m, K);
    } else {
        perm = nullptr;
    }
    k_msm_points<<<(unsigned)((m + MSM_TPB - 1) / MSM_TPB), MSM_TPB, 0, s>>>(pts, scal, P, m, pm, perm, dtab, ptab, K);
}

// Canonical pairwise tree over S segments of m points: for stride 1,2,4,..:
//   T[i] = Ndev(T[i] + T[i+stride]) for i % (2 stride) == 0 and i + stride < m.
// One block folds 256 consecutive points (levels 1..128); out has S*ceil(m/256) entries.
// Level st's pairs (i, i + st), i = 2 st a, go to lanes a = 0, 1, ...: the busy lanes are packed
// into the fewest waves (9 wave-adds per block instead of 27 with lane i taking pair i; the
// same pairs, so the same bits).
__global__ __launch_bounds__(TPB) void k_tree(ge* out, const ge* __restrict__ in, size_t m, int nb) {
    __shared__ ge sh[TPB];
    int seg = blockIdx.x / nb, chunk = blockIdx.x % nb;
    int tid = threadIdx.x;
    size_t base = (size_t)seg * m + (size_t)chunk * TPB;
    int cnt = (int)min((size_t)TPB, m - (size_t)chunk * TPB);
    if (tid < cnt) sh[tid] = in[base + tid];
    __syncthreads();
    for (int st = 1; st < cnt; st <<= 1) {
        const int i = 2 * st * tid;
        if (i + st < cnt) sh[i] = ge_norm_dev(ge_add(sh[i], sh[i + st]));
        __syncthreads();
    }
    if (tid == 0) out[blockIdx.x] = sh[0];
}

void launch_tree(ge* out, const ge* in, int S, size_t m, hipStream_t s) {
    int nb = (int)((m + TPB - 1) / TPB);
    k_tree<<<S * nb, TPB, 0, s>>>(out, in, m, nb);
}

// ------------------------------------------------------------------ verify: challenges & scalars


// range_proof_verify's scalar work (mode 2), one lane per proof: the x challenge
// (challenge.cu:61-77), compute_precise_delta (rp.cu:315-410), enhanced_range_check
// (rp.cu:765-876; called twice at rp.cu:1778/:1785 with the same result), the V match
// (rp.cu:1729-1740) and the polynomial-identity scalars in host-tobytes form (rp.cu:424-435).
// sy = <1^n, y^n> from the caller's power loop (rp.cu:336-343, the same mul/add chain).
__device__ __forceinline__ void prep_std_task(const BatchView& bv, const VerifyWs& ws, const fe* __restrict__ two_i,
                                              size_t p, const fe& z, const fe& z2, const fe& sy) {
    const int n = bv.n;
    sha256_ctx c;
    sha_init(c);
    sha_str(c, "BulletproofXChal");
    sha_fe_canon(c, bv.T1[p].X); sha_fe_canon(c, bv.T1[p].Y);
    sha_fe_canon(c, bv.T2[p].X); sha_fe_canon(c, bv.T2[p].Y);
    sha_str(c, "xcha");                  // memcpy of 4 bytes of "xchal" (challenge.cu:73)
    fe x = challenge_digest(c);
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
    sha256_ctx c;
    // y = H("BulletproofYChal" || V.X V.Y A.X A.Y S.X S.Y || "y_ch")   (challenge.cu:24-44)
    sha_init(c);
    sha_str(c, "BulletproofYChal");
    sha_fe_canon(c, bv.V[p].X); sha_fe_canon(c, bv.V[p].Y);
    sha_fe_canon(c, bv.A[p].X); sha_fe_canon(c, bv.A[p].Y);
    sha_fe_canon(c, bv.S[p].X); sha_fe_canon(c, bv.S[p].Y);
    sha_str(c, "y_ch");
    fe y = challenge_digest(c);
    // z = H("BulletproofZChal" || y || "z_ch")   (challenge.cu:47-58)
    sha_init(c);
    sha_str(c, "BulletproofZChal");
    sha_limbs(c, y.v, 4);
    sha_str(c, "z_ch");
    fe z = challenge_digest(c);
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
            sha256_ctx c;
            sha_init(c);
            sha_str(c, "InnerProductChal");
            sha_limbs(c, tr.v, 4);
            sha_fe_canon(c, bv.L[p * Lr + r].X);
            sha_fe_canon(c, bv.R[p * Lr + r].X);
            u = challenge_digest(c);
            tr = u;
        }
        ws.u[p * Lr + r] = fe_canon(u);
        ws.uinv[p * Lr + r] = fe_canon(fe_invert(u));
    }
    ws.sc[p * 4 + 1] = fe_canon(bv.a[p * abl]);
    ws.sc[p * 4 + 2] = fe_canon(bv.b[p * abl]);
    ws.sc[p * 4 + 3] = fe_canon(bv.c[p]);
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
    sha256_ctx c;
    sha_init(c);
    sha_limbs(c, kx.v, 4); sha_limbs(c, ky.v, 4);
    sha_limbs(c, px.v, 4); sha_limbs(c, py.v, 4);
    fe hs;
    sha_final_limbs(c, hs.v);
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
    sha256_ctx c;
    sha_init(c);
    sha_limbs(c, lx.v, 4); sha_limbs(c, ly.v, 4);
    sha_limbs(c, rx.v, 4); sha_limbs(c, ry.v, 4);
    fe ch;
    sha_final_limbs(c, ch.v);
    ws.chal[p] = ch;
    ws.lr[p * 2] = left;
    ws.lr[p * 2 + 1] = right;
    ws.rflags[p] |= m12 ? 4 : 0;
    if (sd.poly_out) {
        sd.poly_out[p * 4] = left;
        sd.poly_out[p * 4 + 1] = right;
    }
}

// ------------------------------------------------------------------ lane sort (verify)
// Chain length (sm_ops) of the scalar of item j of a per-lane set, read the way the item's
// task reads it (stage0_task / fold_task / final_terms_task).  A lane with no work keys 0.
__device__ __forceinline__ int lane_key(const SlotDev& sd, int kind, int r, size_t j) {
    const BatchView& bv = sd.bv;
    const VerifyWs& ws = sd.ws;
    const size_t B = bv.B;
    const int n = bv.n, Lr = bv.L_len;
    fe s;
    int K = 0;   // the item's prefix-table width (its base is a generator)
    if (kind == SS_STAGE0) {
        size_t i = stage0_class_item(sd, r, (uint32_t)j);
        if (sd.ptab) K = sd.pbits;
        const size_t nA = sd.range_mode ? B * 2 * n : 0, nB = Lr > 0 ? B * 2 * n : 0;
        if (i < nA) {
            size_t seg = i / n, p = seg >> 1;
            s = (seg & 1) ? ws.sH[p * n + i % n] : ws.sG[p];
        } else if (i - nA < nB) {
            i -= nA;
            size_t p = i / (2 * n);
            int grp = (int)(i % (2 * n)) / (n >> 1);
            s = grp < 2 ? ws.uinv[p * Lr] : ws.u[p * Lr];
        } else if (i - nA - nB < 2 * B) {
            i -= nA + nB;
            bool isC = i & 1;
            if (!isC && !sd.range_mode) return 0;
            s = ws.sc[(i >> 1) * 4 + (isC ? 3 : 0)];
        } else {
            i -= nA + nB + 2 * B;
            s = ws.psc[(i / 7) * 8 + i % 7];
            const int k = (int)(i % 7);
            if (k == 2 || k == 5 || k == 6) K = 0;   // V, T1, T2: the proof's own points
        }
    } else if (kind == SS_ROUND) {
        const int np = n >> (r + 1);
        size_t p = j / (4 * np);
        int grp = (int)(j % (4 * np)) / np;
        s = grp < 2 ? ws.uinv[p * Lr + r] : ws.u[p * Lr + r];
    } else {
        s = ws.sc[(j >> 1) * 4 + ((j & 1) ? 2 : 1)];
    }
    return sm_ops_prefix(s, K);
}

__device__ __forceinline__ int lane_set_of(const LaneSortPlan& pl, unsigned b, LaneSortPlan::Set& st) {
    int idx = 0;
    st = pl.set[0];
#pragma unroll
    for (int k = 1; k < LANE_SORT_SETS; k++)
        if (k < pl.count && b >= pl.set[k].block0) { st = pl.set[k]; idx = k; }
    return idx;
}

__global__ __launch_bounds__(LANE_SORT_BLOCK) void k_lane_hist(LaneSortPlan pl, unsigned* bins) {
    __shared__ unsigned h[OPS_BINS];
    for (int k = threadIdx.x; k < OPS_BINS; k += LANE_SORT_BLOCK) h[k] = 0;
    __syncthreads();
    LaneSortPlan::Set st;
    const int si = lane_set_of(pl, blockIdx.x, st);
    const size_t j = (size_t)(blockIdx.x - st.block0) * LANE_SORT_BLOCK + threadIdx.x;
    if (j < st.items) atomicAdd(&h[lane_key(*pl.slot, st.kind, st.r, j)], 1u);
    __syncthreads();
    for (int k = threadIdx.x; k < OPS_BINS; k += LANE_SORT_BLOCK)
        if (h[k]) atomicAdd(&bins[si * OPS_BINS + k], h[k]);
}

// Per set (one block each): longest-first exclusive scan of its bins into offs; bins re-zeroed.
// LANE_SORT_BLOCK (256) threads, LS_PER consecutive scan positions each: a small block gets a CU as
// soon as one block of a running k_terms launch retires there (a 1024-thread block needs a whole
// CU's wave slots and waited for milliseconds behind a concurrent pipeline's stage-0 tick).
constexpr int LS_PER = (OPS_BINS + LANE_SORT_BLOCK - 1) / LANE_SORT_BLOCK;
__global__ __launch_bounds__(LANE_SORT_BLOCK) void k_lane_scan(unsigned* bins, unsigned* offs, int longest_first) {
    __shared__ unsigned wsum[LANE_SORT_BLOCK / 64];
    const int t = threadIdx.x;
    unsigned* bb = bins + (size_t)blockIdx.x * OPS_BINS;
    unsigned v[LS_PER], sum = 0;
#pragma unroll
    for (int u = 0; u < LS_PER; u++) {   // scan position p = LS_PER t + u -> bin k(p)
        const int p = LS_PER * t + u, k = longest_first ? OPS_BINS - 1 - p : p;
        v[u] = p < OPS_BINS ? bb[k] : 0u;
        sum += v[u];
    }
    unsigned inc = sum;   // inclusive scan over the block: waves, then the wave totals
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const unsigned x = __shfl_up(inc, d, 64);
        if ((t & 63) >= d) inc += x;
    }
    if ((t & 63) == 63) wsum[t >> 6] = inc;
    __syncthreads();
    unsigned run = inc - sum;
    for (int w = 0; w < (t >> 6); w++) run += wsum[w];
#pragma unroll
    for (int u = 0; u < LS_PER; u++) {
        const int p = LS_PER * t + u, k = longest_first ? OPS_BINS - 1 - p : p;
        if (p < OPS_BINS) {
            offs[(size_t)blockIdx.x * OPS_BINS + k] = run;
            bb[k] = 0;
        }
        run += v[u];
    }
}

__global__ __launch_bounds__(LANE_SORT_BLOCK) void k_lane_scatter(LaneSortPlan pl, unsigned* offs) {
    __shared__ unsigned cnt[OPS_BINS], base[OPS_BINS];
    for (int k = threadIdx.x; k < OPS_BINS; k += LANE_SORT_BLOCK) cnt[k] = 0;
    __syncthreads();
    LaneSortPlan::Set st;
    const int si = lane_set_of(pl, blockIdx.x, st);
    const size_t j = (size_t)(blockIdx.x - st.block0) * LANE_SORT_BLOCK + threadIdx.x;
    int key = 0;
    unsigned rank = 0;
    if (j < st.items) {
        key = lane_key(*pl.slot, st.kind, st.r, j);
        rank = atomicAdd(&cnt[key], 1u);
    }
    __syncthreads();
    for (int k = threadIdx.x; k < OPS_BINS; k += LANE_SORT_BLOCK)
        if (cnt[k]) base[k] = atomicAdd(&offs[si * OPS_BINS + k], cnt[k]);
    __syncthreads();
    if (j < st.items) st.perm[base[key] + rank] = (uint32_t)j;
}

void launch_lane_sort(const LaneSortPlan& plan, unsigned* bins, unsigned* offs, hipStream_t s) {
    if (!plan.count || !plan.blocks) return;
    k_lane_hist<<<plan.blocks, LANE_SORT_BLOCK, 0, s>>>(plan, bins);
    k_lane_scan<<<plan.count, LANE_SORT_BLOCK, 0, s>>>(bins, offs, plan.longest_first);
    k_lane_scatter<<<plan.blocks, LANE_SORT_BLOCK, 0, s>>>(plan, offs);
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
#ifdef BP_TERMS_WPE   // A/B: a register budget for more waves per SIMD than k_terms runs (room for other kernels' waves)
#define BP_TERMS_BOUNDS __launch_bounds__(TPB) __attribute__((amdgpu_waves_per_eu(BP_TERMS_WPE, 8)))
#else
#define BP_TERMS_BOUNDS __launch_bounds__(TPB, BP_TERMS_OCC)
#endif
template <int QL>
__global__ BP_TERMS_BOUNDS void k_terms(RegionList rl, const SlotDev* __restrict__ slots,
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
        if (sd.range_mode && l < B) prep_range_task(sd.bv, sd.ws, two_i, l, sd.range_mode);
        else prep_ipa_task(sd.bv, sd.ws, sd.range_mode ? l - B : l);
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

static inline unsigned nblk(size_t items) { return (unsigned)((items + TPB - 1) / TPB); }

void launch_terms(const RegionList& rl, const SlotDev* slots, const ge* G, const ge* H, const ge* g, const ge* h,
                  const ge* dtab, const fe* two_i, hipStream_t s, int ql) {
    if (!rl.total) return;
    // A/B knob: unused dynamic LDS per block, to cap how many k_terms blocks share a CU
    static const unsigned pad = [] { const char* e = getenv("HIPBP_TERMS_LDS_PAD"); return e ? (unsigned)atoi(e) : 0u; }();
    if (ql == 16) k_terms<16><<<nblk(rl.total), TPB, pad, s>>>(rl, slots, G, H, g, h, dtab, two_i);
    else if (ql == 4) k_terms<4><<<nblk(rl.total), TPB, pad, s>>>(rl, slots, G, H, g, h, dtab, two_i);
    else if (ql == 2) k_terms<2><<<nblk(rl.total), TPB, pad, s>>>(rl, slots, G, H, g, h, dtab, two_i);
    else k_terms<1><<<nblk(rl.total), TPB, pad, s>>>(rl, slots, G, H, g, h, dtab, two_i);
}


// ------------------------------------------------------------------ batch field ops
// cuda_field_ops.cu:37-73 (add/sub/mul), :147 (square quirk), :521 (SoA add: limbwise, no carry)
__global__ __launch_bounds__(TPB) void k_field_op(int op, fe* r, const fe* __restrict__ a, const fe* __restrict__ b,
                                                  size_t count) {
    size_t i = gid();
    if (i >= count) return;
    fe x = a[i], y;
    if (op != 3 && op != 7) y = b[i];   // unary ops take no b
    fe z;
    switch (op) {
        case 0: z = fe_add(x, y); break;
        case 1: z = fe_sub(x, y); break;
        case 2: z = fe_mul(x, y); break;
        case 3: z = fe_square_kernel_quirk(x); break;
        case 6: {   // the product fold alone on t = a || b (fe25519_mul's reduction, for its KATs)
            uint64_t t[8] = {x.v[0], x.v[1], x.v[2], x.v[3], y.v[0], y.v[1], y.v[2], y.v[3]};
            z = fe_fold512(t);
            break;
        }
        case 7: z = fe_sq(x); break;   // fe25519_sq (dedicated squaring; == mul(x, x))
        case 8:                         // fe_addsub's sum / difference (the drain forms' fused
        case 9: {                       // block: its rare-edge path is tested through these)
            fe sm, df;
            fe_addsub(x, y, sm, df);
            z = op == 8 ? sm : df;
            break;
        }
        default:
#pragma unroll
            for (int k = 0; k < 4; k++) z.v[k] = x.v[k] + y.v[k];
            break;
    }
    r[i] = z;
}

void launch_field_op(int op, fe* r, const fe* a, const fe* b, size_t count, hipStream_t s) {
    if (count == 0) return;
    k_field_op<<<nblk(count), TPB, 0, s>>>(op, r, a, b, count);
}


// The halving tree's levels with stride <= 32 (their pairs (t, t+st) lie inside wave 0), in
// registers: lane t takes lane t+st's value over a wave shuffle and adds it when t < st and
// t + st < lim — exactly the LDS tree's pairs, order and guard.
__device__ __forceinline__ fe fe_wave_tail(fe v, int tid, unsigned st, size_t lim) {
    for (; st > 0; st >>= 1) {
        fe o;
#pragma unroll
        for (int i = 0; i < 4; i++) {
            uint32_t lo = (uint32_t)__shfl_down((int)(uint32_t)v.v[i], st, 64);
            uint32_t hi = (uint32_t)__shfl_down((int)(uint32_t)(v.v[i] >> 32), st, 64);
            o.v[i] = (uint64_t)lo | ((uint64_t)hi << 32);
        }
        if (tid < (int)st && (size_t)(tid + st) < lim) v = fe_add(v, o);
    }
    return v;
}

// ------------------------------------------------------------------ field inner products
// cuda_inner_product.cu:154-183 field_vector_inner_product_shared_kernel, one block of
// nthreads = min(n, 512): products, then halving tree from nthreads/2 with tid+stride < n.
__global__ __launch_bounds__(512) void k_ip_shared(fe* out, const fe* __restrict__ a, const fe* __restrict__ b,
                                                   size_t n) {
    __shared__ fe sh[512];
    int tid = threadIdx.x;
    sh[tid] = fe_mul(a[tid], b[tid]);
    __syncthreads();
    unsigned st = blockDim.x / 2;
    for (; st > 32; st >>= 1) {
        if (tid < (int)st && (size_t)(tid + st) < n) sh[tid] = fe_add(sh[tid], sh[tid + st]);
        __syncthreads();
    }
    if (tid < 64) {
        fe v = sh[tid];
        v = fe_wave_tail(v, tid, st, n);
        if (tid == 0) *out = v;
    }
}

// cuda_inner_product.cu:33-61 field_vector_inner_product_kernel: grid-stride fold from 0,
// then block tree 128..1 over all 256 slots.  With `warp_tail` the reference stops the block tree
// at 32 and warp_reduce_field_element (:219-257) does 16..1 (batch_inner_product_kernel :260-299):
// the same strides, so both run the wave-shuffle tail below 64.  blockIdx.y selects the vector
// (stride n) for the batched form.
__global__ __launch_bounds__(TPB) void k_ip_grid(fe* out, const fe* __restrict__ a, const fe* __restrict__ b,
                                                 size_t n, size_t grid_threads, int warp_tail) {
    (void)warp_tail;
    __shared__ fe sh[TPB];
    int tid = threadIdx.x;
    size_t vec = blockIdx.y;
    a += vec * n;
    b += vec * n;
    fe acc = fe_set(0);
    for (size_t idx = (size_t)blockIdx.x * TPB + tid; idx < n; idx += grid_threads) acc = fe_add(acc, fe_mul(a[idx], b[idx]));
    sh[tid] = acc;
    __syncthreads();
    unsigned st = TPB / 2;
    for (; st > 32; st >>= 1) {
        if (tid < (int)st) sh[tid] = fe_add(sh[tid], sh[tid + st]);
        __syncthreads();
    }
    if (tid < 64) {
        fe v = sh[tid];
        v = fe_wave_tail(v, tid, st, TPB);
        if (tid == 0) out[vec * gridDim.x + blockIdx.x] = v;
    }
}

// cuda_inner_product.cu:69-92 fe25519_reduce_kernel: 256 slots, partials beyond 256 unread.
__global__ __launch_bounds__(TPB) void k_ip_reduce(fe* out, const fe* __restrict__ part, size_t np) {
    __shared__ fe sh[TPB];
    int tid = threadIdx.x;
    sh[tid] = (size_t)tid < np ? part[tid] : fe_set(0);
    __syncthreads();
    unsigned st = TPB / 2;
    for (; st > 32; st >>= 1) {
        if (tid < (int)st && (size_t)(tid + st) < np) sh[tid] = fe_add(sh[tid], sh[tid + st]);
        __syncthreads();
    }
    if (tid < 64) {
        fe v = sh[tid];
        v = fe_wave_tail(v, tid, st, np);
        if (tid == 0) *out = v;
    }
}

void launch_ip_shared(fe* out, const fe* a, const fe* b, size_t n, hipStream_t s) {
    unsigned nt = (unsigned)(n < 512 ? n : 512);
    if (nt == 0) return;
    k_ip_shared<<<1, nt, 0, s>>>(out, a, b, n);
}

void launch_ip_grid(fe* out, fe* part, const fe* a, const fe* b, size_t n, hipStream_t s) {
    size_t nb = (n + TPB - 1) / TPB;
    if (nb > 1024) nb = 1024;
    k_ip_grid<<<dim3((unsigned)nb, 1), TPB, 0, s>>>(part, a, b, n, nb * TPB, 0);
    k_ip_reduce<<<1, TPB, 0, s>>>(out, part, nb);
}

// Batched form: the reference launches min(1024, ceil(n/256)) x-blocks per vector that all
// write results[vec] (a race when n > 256); block 0's value is one of its possible outcomes
// and is the one returned.
void launch_ip_batch(fe* out, const fe* a, const fe* b, size_t n, size_t nvec, hipStream_t s) {
    size_t nb = (n + TPB - 1) / TPB;
    if (nb > 1024) nb = 1024;
    if (nb == 0) nb = 1;
    k_ip_grid<<<dim3(1, (unsigned)nvec), TPB, 0, s>>>(out, a, b, n, nb * TPB, 1);
}

// elementwise host invert chain (defined semantics for cuda_batch_field_invert)
__global__ __launch_bounds__(TPB) void k_invert(fe* r, const fe* __restrict__ a, size_t count) {
    size_t i = gid();
    if (i < count) r[i] = fe_invert(a[i]);
}
void launch_invert(fe* r, const fe* a, size_t count, hipStream_t s) {
    if (count) k_invert<<<nblk(count), TPB, 0, s>>>(r, a, count);
}

// Generic canonical-tree MSM on device: ptsbuf holds n points, part0/part1 ping-pong.
// Canonical tree over n points (levels 1, 2, 4, ...: one k_tree launch per 256x reduction).
void launch_tree_full(ge* result, const ge* in, size_t n, ge* part0, ge* part1, hipStream_t s, int S) {
    size_t m = n;
    ge* bufs[2] = {part0, part1};
    int w = 0;
    while (true) {
        size_t nb = (m + TPB - 1) / TPB;
        ge* out = (nb == 1) ? result : bufs[w];
        launch_tree(out, in, S, m, s);
        if (nb == 1) break;
        in = out;
        m = nb;
        w ^= 1;
    }
}

void launch_msm_full(ge* result, const fe* scal, const ge* P, size_t n, ge* ptsbuf, ge* part0, ge* part1,
                     uint32_t* perm, unsigned* bins, const ge* dtab, hipStream_t s, size_t count, const ge* ptab,
                     int K) {
    // count MSMs of n points each over the same points: one per-point launch over all count*n
    // items (chain-length sorted together), then the canonical tree per segment
    launch_msm_points(ptsbuf, scal, P, n * count, perm, bins, dtab, s, n, ptab, K);
    launch_tree_full(result, ptsbuf, n, part0, part1, s, (int)count);
}

}  // namespace bp
