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
// (dtab, the identity-doubling table, and two_i are built on the host: bp_capi.hip Engine::init)
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

static inline unsigned nblk(size_t items) { return (unsigned)((items + TPB - 1) / TPB); }

void launch_terms(const RegionList& rl, const SlotDev* slots, const ge* G, const ge* H, const ge* g, const ge* h,
                  const ge* dtab, const fe* two_i, hipStream_t s, int ql) {
    if (!rl.total) return;
    // A/B knob: unused dynamic LDS per block, to cap how many k_terms blocks share a CU
    static const unsigned pad = [] { const char* e = getenv("HIPBP_TERMS_LDS_PAD"); return e ? (unsigned)atoi(e) : 0u; }();
    if (ql == 16) launch_terms16(rl, slots, G, H, g, h, dtab, two_i, s, pad);
    else if (ql == 4) launch_terms4(rl, slots, G, H, g, h, dtab, two_i, s, pad);
    else if (ql == 2) launch_terms2(rl, slots, G, H, g, h, dtab, two_i, s, pad);
    else launch_terms1(rl, slots, G, H, g, h, dtab, two_i, s, pad);
}


// ------------------------------------------------------------------ batch field ops
// cuda_field_ops.cu:37-73 (add/sub/mul), :147 (square quirk), :521 (SoA add: limbwise, no carry)
__global__ __launch_bounds__(TPB) void k_field_op(int op, fe* r, const fe* __restrict__ a, const fe* __restrict__ b,
                                                  size_t count) {
    size_t i = gid();
    if (op == 10 || op == 12) {   // the drain forms' quad-split products fe_mul_q4 / fe_mul_q4_k (by k):
        i >>= 2;                  // element i >> 2 on lane quad i >> 2 (a whole quad leaves together:
        if (i >= count) return;   // the DPP sums stay inside live quads)
        const fe z = op == 10 ? fe_mul_q4(a[i], b[i]) : fe_mul_q4_k(a[i]);
        if ((threadIdx.x & 3) == 0) r[i] = z;
        return;
    }
    if (i >= count) return;
    fe x = a[i], y;
    if (op != 3 && op != 7 && op != 11) y = b[i];   // unary ops take no b
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
        case 11: z = fe_mul_k(x); break;   // fe25519_mul(x, k), the point operations' product by k
        case 8:                         // fe_addsub's sum / difference (the drain forms' fused
        case 9: {                       // block: its rare-edge path is tested through these)
            fe sm, df;
            fe_addsub(x, y, sm, df);
            z = op == 8 ? sm : df;
            break;
        }
        // the row step's latency forms (LAT 1: field_asm.h *_lat) and its deferred forms (LAT 2:
        // *_lat_acc, the fast statement alone; here per element, as sm_row does per step: when the
        // running max of the test words is 2^32-1 the exact-capable form recomputes the result)
        case 13: z = fe_add<1>(x, y); break;
        case 14: {
            uint32_t acc = 0;
            z = fe_add<2>(x, y, &acc);
            if (acc == 0xFFFFFFFFu) z = fe_add<1>(x, y);
            break;
        }
        case 15:
        case 16: {
            fe sm, df;
            fe_addsub<1>(x, y, sm, df);
            z = op == 15 ? sm : df;
            break;
        }
        case 17:
        case 18: {
            fe sm, df;
            uint32_t acc = 0;
            fe_addsub<2>(x, y, sm, df, &acc);
            if (acc == 0xFFFFFFFFu) fe_addsub<1>(x, y, sm, df);
            z = op == 17 ? sm : df;
            break;
        }
        case 19:
        case 20: {
            uint64_t t[8] = {x.v[0], x.v[1], x.v[2], x.v[3], y.v[0], y.v[1], y.v[2], y.v[3]};
            if (op == 19) {
                z = fe_fold512<1>(t);
            } else {
                uint32_t acc = 0;
                z = fe_fold512<2>(t, &acc);
                if (acc == 0xFFFFFFFFu) z = fe_fold512<1>(t);
            }
            break;
        }
        default:
#pragma unroll
            for (int k = 0; k < 4; k++) z.v[k] = x.v[k] + y.v[k];
            break;
    }
    r[i] = z;
}

// The challenge path's SHA-256 message shapes (sha256_dev.h), one per lane, for the device-vs-FIPS
// check (hipbp_sha_probe, tests/test_gpu_parity.py): item i reads six field elements in[6i..6i+5]
// (a point's X, Y pairs for the shapes that hash points).
__global__ __launch_bounds__(TPB) void k_sha_probe(int kind, fe* out, const fe* __restrict__ in, size_t count) {
    const size_t i = gid();
    if (i >= count) return;
    const fe* f = in + i * 6;
    auto pt = [&](int k) { return ge{f[k], f[k + 1], fe_set(1), fe_set(0)}; };
    fe r;
    switch (kind) {
        case 0: r = chal_y(pt(0), pt(2), pt(4)); break;          // challenge.cu:24-44
        case 1: r = chal_z(f[0]); break;                          // challenge.cu:47-58
        case 2: r = chal_x(pt(0), pt(2)); break;                  // challenge.cu:61-77
        case 3: r = chal_ip(f[0], f[1], f[2]); break;             // crv:185-205
        case 4: r = chal_ip_start(f[0], f[1], f[2]); break;       // rp.cu:1636-1650
        default: r = sha_4fe(f[0], f[1], f[2], f[3]); break;      // crv:330-344, rp.cu:560-566
    }
    out[i] = r;
}

void launch_sha_probe(int kind, fe* out, const fe* in, size_t count, hipStream_t s) {
    if (count == 0) return;
    k_sha_probe<<<nblk(count), TPB, 0, s>>>(kind, out, in, count);
}

void launch_field_op(int op, fe* r, const fe* a, const fe* b, size_t count, hipStream_t s) {
    if (count == 0) return;
    k_field_op<<<nblk(op == 10 || op == 12 ? 4 * count : count), TPB, 0, s>>>(op, r, a, b, count);
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
