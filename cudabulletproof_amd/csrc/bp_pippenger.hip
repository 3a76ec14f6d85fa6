// bp_pippenger.hip — Pippenger bucket MSM (BASELINE configs[2]: "Pippenger, window=12") over the
// reference's fe25519/ge25519 arithmetic.  A labelled alternative to the graded MSM (SURVEY §7,
// §8(d) config 3): the reference's own MSM result comes from per-point double-and-add plus the
// canonical tree (A9), and its arithmetic is not associative, so no regrouping reproduces those
// bits.  This computes the bucket algorithm that the tests restate in C (orc_msm_pippenger)
// bit for bit — every grouping below is fixed, none depends on scheduling:
//
//   digit_w(i) = bits [c w, c w + c) of s_i;  B_{w,b} = pairwise tree over the points of bucket b
//   in index order;  chunk k of M = 16 buckets: running sums R, S, then V = S + (kM) R;
//   S_w = pairwise tree over the chunks;  T = Horner over the windows (c doublings + add).
//
// GPU mapping.  (1) one (key = digit, value = w n + i) pair per window and point, generated
// window-major, stable radix sort (rocPRIM, 16-bit keys, values from a counting iterator) on the
// digit bits -> each bucket's points contiguous in index order; bucket bounds from the sorted
// pairs (no atomics).  (2) the bucket trees level by level over ALL buckets at once: a level's
// lane takes one adjacent pair of one bucket's current list (lists compacted and padded to even
// length after every level, offsets by an exclusive scan), so every lane of every wave adds —
// ~W n point additions at the VALU roof instead of one lane walking a bucket.  (3) one lane per
// chunk (W 2^c / 16 lanes) for the running sums and the small scalar-mult, (4) one block per
// window: the chunk tree in LDS, (5) one lane quad: the Horner chain (~256 doublings,
// latency-bound), on a side stream so its top-half part overlaps the bottom half's buckets.
// The host never waits: the tree depth is read on the device (pip_steps), so independent MSMs
// on different streams overlap one's latency-bound chains with another's bucket trees.
#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/iterator/counting_iterator.hpp>

#include <algorithm>
#include <cstdlib>
#include <map>
#include <mutex>

#include "bp_kernels.h"
#include "ge25519_dev.h"
#include "ge25519_quad.h"

namespace bp {

namespace {
constexpr int PTPB = 256;
constexpr int PM = 16;   // buckets per chunk

// Division of 32-bit values by a run-time invariant d >= 1 (round-up multiplier, Granlund and
// Montgomery): q = (t + ((x - t) >> s1)) >> s2 with t = umulhi(m, x), exact for every 32-bit x.
struct FastDiv {
    uint32_t d, m;
    int s1, s2;
};
inline FastDiv fastdiv_make(uint32_t d) {
    int l = 0;
    while (l < 32 && (1ull << l) < d) l++;
    FastDiv f;
    f.d = d;
    f.m = (uint32_t)((((1ull << l) - d) << 32) / d + 1);
    f.s1 = l < 1 ? l : 1;
    f.s2 = l > 1 ? l - 1 : 0;
    return f;
}
__device__ __forceinline__ uint32_t fdiv(uint32_t x, const FastDiv& f) {
    const uint32_t t = __umulhi(f.m, x);
    return (t + ((x - t) >> f.s1)) >> f.s2;
}

// Sort input: element g = v n + i (virtual window v = m Wp + lw: MSM m of the batch, window
// lw = w - w0 of the part, point i), generated window-major, so a STABLE sort on the digit leaves
// each bucket (v, d) contiguous and in index order (buckets in digit-major order).  Two key forms:
//  * 32-bit keys (when c + ib <= 32, ib = bits of n - 1): key = digit << ib | i, sorted on bits
//    [ib, ib + c) with no values; the sorted key itself names the point.
//  * 16-bit keys otherwise: key = the digit, value = g (a counting iterator, never stored); the
//    bucket of a sorted element is ((g / n) << c) | digit.
// MSM m's scalars are s[m n .. m n + n); all share the points.  One thread per V scalars (m, i..):
// it reads them once and writes their Wp keys, each store coalesced over consecutive i.
// It also zeroes the bucket counts cnt[0 .. nb) and the three words (longest list, bidfill and tail
// queue lengths) that the histogram, k_pip_len0 and k_pip_lay_part accumulate into (no memset
// launches on the serial path).
template <int V, typename KT>   // V > 1 needs n % V == 0 (one V-key store per window)
__global__ __launch_bounds__(PTPB) void k_pip_keys(const fe* __restrict__ s, FastDiv fn, uint32_t count, int c,
                                                  int ib, int w0, int Wp, KT* keys, uint32_t* cnt, size_t nb,
                                                  unsigned* maxlen) {
    const size_t tid = (size_t)blockIdx.x * PTPB + threadIdx.x;
    for (size_t b = tid; b < nb; b += (size_t)gridDim.x * PTPB) cnt[b] = 0;
    if (tid < 3) maxlen[tid] = 0;   // [0] the longest list, [1] k_pip_bidfill's queue length, [2] k_pip_tail's
    const uint32_t n = fn.d, g = (uint32_t)tid * V;
    if (g >= count * n) return;
    const uint32_t m = fdiv(g, fn), i = g - m * n;
    // each scalar as a 256-bit shift register, shifted right by c per window (a limb index that
    // varies with the window would put the scalars in scratch)
    fe sc[V];
#pragma unroll
    for (int u = 0; u < V; u++) sc[u] = s[g + u];
    auto shr = [&](fe& x) {
        x.v[0] = (x.v[0] >> c) | (x.v[1] << (64 - c));
        x.v[1] = (x.v[1] >> c) | (x.v[2] << (64 - c));
        x.v[2] = (x.v[2] >> c) | (x.v[3] << (64 - c));
        x.v[3] >>= c;
    };
    for (int k = 0; k < w0; k++)
#pragma unroll
        for (int u = 0; u < V; u++) shr(sc[u]);
    const uint64_t mask = (1ull << c) - 1;
    KT* out = keys + (size_t)m * Wp * n + i;
    for (int lw = 0; lw < Wp; lw++) {
        // bits [c (w0 + lw), + c) of the 256-bit scalar (zeros past bit 255)
        uint32_t d[V];
#pragma unroll
        for (int u = 0; u < V; u++) {
            d[u] = (uint32_t)(sc[u].v[0] & mask);
            if constexpr (sizeof(KT) == 4) d[u] = (d[u] << ib) | (i + u);
            shr(sc[u]);
        }
        KT* o = out + (size_t)lw * n;
        if constexpr (V == 4 && sizeof(KT) == 2) {
            *(uint64_t*)o = (uint64_t)d[0] | ((uint64_t)d[1] << 16) | ((uint64_t)d[2] << 32) | ((uint64_t)d[3] << 48);
        } else if constexpr (V == 4) {
            *(uint4*)o = make_uint4(d[0], d[1], d[2], d[3]);
        } else {
            o[0] = (KT)d[0];
        }
    }
}

__device__ __forceinline__ uint32_t pip_bucket(const uint16_t* __restrict__ keys, const uint32_t* __restrict__ vals,
                                               size_t p, const FastDiv& fn, int c) {
    return (fdiv(vals[p], fn) << c) | keys[p];
}

// Bucket sizes straight from the unsorted keys (the sort only orders them): a block takes a tile
// of one virtual window's keys, counts the digits in LDS and adds its counts to cnt[(v << c) | d].
// 1024 threads per block and four 16-byte loads in flight per thread: the loop is bound by load
// latency, not by the LDS atomics.
constexpr uint32_t HIST_TILE = 65536;
constexpr int HIST_TPB = 1024;
template <typename KT>
__global__ __launch_bounds__(HIST_TPB) void k_pip_hist(const KT* __restrict__ keys, uint32_t n, int c, int ib,
                                                      uint32_t tpw, uint32_t* cnt) {
    extern __shared__ uint32_t h[];
    const uint32_t NB = 1u << c, v = blockIdx.x / tpw, t = blockIdx.x - v * tpw;
    for (uint32_t d = threadIdx.x; d < NB; d += HIST_TPB) h[d] = 0;
    __syncthreads();
    const KT* __restrict__ k = keys + (size_t)v * n;
    const uint32_t s0 = t * HIST_TILE, e = (t + 1) * HIST_TILE < n ? (t + 1) * HIST_TILE : n;
    bool vec = false;
    if constexpr (sizeof(KT) == 4) {
        vec = (n & 3) == 0;
        if (vec) {   // rows and tiles start 16-byte aligned; e - s0 is a multiple of 4
            const uint4* __restrict__ k4 = (const uint4*)(k + s0);
            const uint32_t n4 = (e - s0) >> 2;
            for (uint32_t j = threadIdx.x; j < n4; j += 4 * HIST_TPB) {
                uint4 a[4];
#pragma unroll
                for (int u = 0; u < 4; u++)
                    if (j + u * HIST_TPB < n4) a[u] = k4[j + u * HIST_TPB];
#pragma unroll
                for (int u = 0; u < 4; u++)
                    if (j + u * HIST_TPB < n4) {
                        atomicAdd(&h[a[u].x >> ib], 1u);
                        atomicAdd(&h[a[u].y >> ib], 1u);
                        atomicAdd(&h[a[u].z >> ib], 1u);
                        atomicAdd(&h[a[u].w >> ib], 1u);
                    }
            }
        }
    }
    if (!vec)
        for (uint32_t j = s0 + threadIdx.x; j < e; j += HIST_TPB) atomicAdd(&h[(uint32_t)k[j] >> ib], 1u);
    __syncthreads();
    for (uint32_t d = threadIdx.x; d < NB; d += HIST_TPB)
        if (h[d]) atomicAdd(&cnt[((size_t)v << c) | d], h[d]);
}

// Bucket lists are processed two tree levels per launch ("steps"): a step's lane takes one
// aligned group of 4 consecutive elements of one bucket's current list and reduces it exactly as
// levels s and 2s of the pairwise tree do (x0+x1, x2+x3, then their sum; a short last group
// carries), so lists are padded to a multiple of 4.  bid[pos] = the bucket of element pos (every
// group head is a real element, so no search is needed).  k_pip_len0: the longest list (one atomic per wave), and the counts in sorted order — digit-major, virtual
// window minor — whose exclusive scan is each bucket's start in the sorted array.
constexpr uint32_t BID_PIECE = 4096;   // list elements per k_pip_bidfill wave
__global__ __launch_bounds__(PTPB) void k_pip_len0(const uint32_t* __restrict__ len, uint32_t* cnt_t,
                                                  size_t nb, int c, uint32_t Wv, unsigned* maxlen, ge* S,
                                                  uint2* bq) {
    const size_t b = (size_t)blockIdx.x * PTPB + threadIdx.x;
    uint32_t L = 0;
    if (b < nb) {
        L = len[b];
        cnt_t[(b & ((1u << c) - 1)) * Wv + (b >> c)] = L;
        if (!L) S[b] = ge_zero();   // an empty bucket's sum (the steps write every other one)
        // a long list's pieces past the first go to k_pip_bidfill's extra waves (maxlen[1]
        // counts them; at most N / BID_PIECE in all)
        if (L > BID_PIECE) {
            const uint32_t np = (L - 1) / BID_PIECE, q = atomicAdd(&maxlen[1], np);
            for (uint32_t u = 0; u < np; u++) bq[q + u] = make_uint2((uint32_t)b, u + 1);
        }
    }
#pragma unroll
    for (int d = 32; d > 0; d >>= 1) {
        const uint32_t o = __shfl_xor(L, d, 64);
        L = o > L ? o : L;
    }
    // same-address atomics serialize: one per block (the block's waves meet in LDS), and none
    // where a plain read already shows it cannot raise the maximum
    __shared__ uint32_t wmax[PTPB / 64];
    if ((threadIdx.x & 63) == 0) wmax[threadIdx.x >> 6] = L;
    __syncthreads();
    if (threadIdx.x == 0) {
#pragma unroll
        for (int w = 1; w < PTPB / 64; w++) L = wmax[w] > L ? wmax[w] : L;
        if (L > __atomic_load_n(maxlen, __ATOMIC_RELAXED)) atomicMax(maxlen, L);
    }
}
__global__ __launch_bounds__(PTPB) void k_pip_start(const uint32_t* __restrict__ start_t, size_t nb, int c, uint32_t Wv,
                                                   uint32_t* start) {
    const size_t b = (size_t)blockIdx.x * PTPB + threadIdx.x;
    if (b < nb) start[b] = start_t[(b & ((1u << c) - 1)) * Wv + (b >> c)];
}

// Tree steps needed for the longest bucket list (levels = ceil(log2 maxlen), at least 1; two
// levels per step).  Every step kernel reads it on the device, so the host never waits for the
// bucket-size histogram: it launches the worst-case number of steps (lists are at most n long)
// and the steps past the data's depth exit at once.
__device__ __forceinline__ int pip_steps(const unsigned* maxlen) {
    const unsigned m = *maxlen;
    int levels = 1;
    while (levels < 31 && (1u << levels) < m) levels++;
    return (levels + 1) / 2;
}

// Every step's layout at once.  A list of length L is finished by its step when L <= 4 (its sum
// goes to S[b]); otherwise the step leaves ceil(L / 4) elements.  So layout t of every bucket
// follows from the bucket sizes alone: LEN_t[b], PAD_t[b] = LEN_t[b] padded to x4, and
// OFF_t = the exclusive scan of PAD_t over the buckets.  Two launches form all T layers (the
// per-step scans were two launches per step on the bucket trees' critical path), one block row
// per layer (blockIdx.y): k_pip_lay_part writes LEN/PAD for SCAN_PER consecutive buckets per
// thread and one partial sum per block; k_pip_lay_fin adds the partial sums of the blocks before
// it and scans.
constexpr int SCAN_PER = 4;
constexpr int SCAN_BLK = PTPB * SCAN_PER;

__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t u = __shfl_up(v, d, 64);
        if (lane >= d) v += u;
    }
    return v;
}

// The extra layer T (the last block row) scans the bucket sizes in sorted order instead (cnt_t:
// digit-major, virtual window minor, unpadded): OFF_T is each bucket's start in the sorted array.
// Layer TT (TT < T; TT = 0: none) also queues every bucket whose list there needs more than one
// more step (LEN_TT > 4) for k_pip_tail: tailq[0 .. *tailn); step TT finishes the others.
__global__ __launch_bounds__(PTPB) void k_pip_lay_part(const uint32_t* __restrict__ len0,
                                                      const uint32_t* __restrict__ cnt_t, int T, size_t nb,
                                                      uint32_t* LEN, uint32_t* PAD, uint32_t* part, unsigned nparts,
                                                      int TT, uint32_t* tailq, unsigned* tailn) {
    __shared__ uint32_t wsum[PTPB / 64];
    const int t = blockIdx.y;   // layer
    const size_t b0 = (size_t)blockIdx.x * SCAN_BLK + (size_t)threadIdx.x * SCAN_PER;
    uint32_t sum = 0;
#pragma unroll
    for (int k = 0; k < SCAN_PER; k++) {
        if (b0 + k < nb && t == T) {
            const uint32_t L = cnt_t[b0 + k];
            PAD[(size_t)t * nb + b0 + k] = L;
            sum += L;
        } else if (b0 + k < nb) {
            uint32_t L = len0[b0 + k];
            for (int u = 0; u < t; u++) L = L <= 4 ? 0u : (L + 3) >> 2;
            const uint32_t pd = (L + 3) & ~3u;
            if (TT && t == TT && L > 4) tailq[atomicAdd(tailn, 1u)] = (uint32_t)(b0 + k);
            LEN[(size_t)t * nb + b0 + k] = L;
            PAD[(size_t)t * nb + b0 + k] = pd;
            sum += pd;
        }
    }
    const uint32_t inc = wave_incl_scan(sum);
    if ((threadIdx.x & 63) == 63) wsum[threadIdx.x >> 6] = inc;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t tot = 0;
#pragma unroll
        for (int w = 0; w < PTPB / 64; w++) tot += wsum[w];
        part[(size_t)t * nparts + blockIdx.x] = tot;
    }
}

__global__ __launch_bounds__(PTPB) void k_pip_lay_fin(const uint32_t* __restrict__ PAD, const uint32_t* __restrict__ part,
                                                     unsigned nparts, size_t nb, uint32_t* OFF) {
    __shared__ uint32_t wsum[PTPB / 64];
    __shared__ uint32_t pre;
    const int t = blockIdx.y;   // layer
    const size_t b0 = (size_t)blockIdx.x * SCAN_BLK + (size_t)threadIdx.x * SCAN_PER;
    if (threadIdx.x < 64) {   // sum of layer t's partial sums of the blocks before this one
        uint32_t v = 0;
        for (unsigned i = threadIdx.x; i < blockIdx.x; i += 64) v += part[(size_t)t * nparts + i];
        v = wave_incl_scan(v);
        if (threadIdx.x == 63) pre = v;
    }
    uint32_t p[SCAN_PER], sum = 0;
#pragma unroll
    for (int k = 0; k < SCAN_PER; k++) {
        p[k] = b0 + k < nb ? PAD[(size_t)t * nb + b0 + k] : 0u;
        sum += p[k];
    }
    const uint32_t inc = wave_incl_scan(sum);
    if ((threadIdx.x & 63) == 63) wsum[threadIdx.x >> 6] = inc;
    __syncthreads();
    uint32_t run = pre + inc - sum;
    for (int w = 0; w < (int)(threadIdx.x >> 6); w++) run += wsum[w];
#pragma unroll
    for (int k = 0; k < SCAN_PER; k++) {
        if (b0 + k < nb) OFF[(size_t)t * nb + b0 + k] = run;
        run += p[k];
    }
}

__global__ __launch_bounds__(PTPB) void k_pip_bid0(const uint16_t* __restrict__ keys, const uint32_t* __restrict__ vals,
                                                  size_t N, FastDiv fn, int c, const uint32_t* __restrict__ start,
                                                  const uint32_t* __restrict__ off, uint32_t* bid) {
    const size_t p = (size_t)blockIdx.x * PTPB + threadIdx.x;
    if (p >= N) return;
    const uint32_t b = pip_bucket(keys, vals, p, fn, c);
    bid[off[b] + (p - start[b])] = b;
}

// 32-bit-key path: bid from the layout alone (no sorted value says which virtual window an element
// is in).  A wave writes one BID_PIECE-element piece of one bucket's list, at its group heads
// only (step 0 reads bid only there: every head is a multiple of 4): wave w < nb takes bucket w's
// first piece, wave nb + q the q-th entry of k_pip_len0's queue of further pieces, so the deep
// buckets (the top window's few digits) do not leave one wave looping over a whole list.
__global__ __launch_bounds__(PTPB) void k_pip_bidfill(const uint32_t* __restrict__ len, const uint32_t* __restrict__ off,
                                                     size_t nb, const unsigned* __restrict__ maxlen,
                                                     const uint2* __restrict__ bq, uint32_t* bid) {
    const size_t w = ((size_t)blockIdx.x * PTPB + threadIdx.x) >> 6;
    uint32_t b, pc = 0;
    if (w < nb) {
        b = (uint32_t)w;
    } else {
        if (w - nb >= maxlen[1]) return;
        const uint2 e = bq[w - nb];
        b = e.x;
        pc = e.y;
    }
    const uint32_t L = len[b], o = off[b];
    const uint32_t e = L < (pc + 1) * BID_PIECE ? L : (pc + 1) * BID_PIECE;
    for (uint32_t j = pc * BID_PIECE + 4 * (threadIdx.x & 63); j < e; j += 256) bid[o + j] = b;
}

// (min 4 waves per SIMD: the compiler keeps it at 128 VGPRs)

// Bucket-tree step: each lane reduces one aligned 4-element group of a bucket's list (2 levels).
// When few groups remain (the deep buckets' tail steps, a wave-uniform test on the device-side
// count), each group takes a lane octet instead: quads A and B add elements (0, 1) and (2, 3) side
// by side on ge_op_quad, then A adds B's sum, moved over DPP: 2 point-op latencies instead of
// 3 adds on one lane.  The same adds in the same order, so the same bits.
__global__ __launch_bounds__(PTPB, 4) void k_pip_step(int t, const unsigned* __restrict__ maxlen, const ge* __restrict__ P,
                                                  FastDiv fn, const uint32_t* __restrict__ keys32, uint32_t imask,
                                                  const uint32_t* __restrict__ vals,
                                                  const uint32_t* __restrict__ start, const ge* __restrict__ Qin,
                                                  const uint32_t* __restrict__ bid, const uint32_t* __restrict__ off,
                                                  const uint32_t* __restrict__ len, const uint32_t* __restrict__ pad,
                                                  const uint32_t* __restrict__ off2, ge* Qout, uint32_t* bid2,
                                                  ge* S, size_t nb, size_t lanes, int tail_t) {
    const size_t k = (size_t)blockIdx.x * PTPB + threadIdx.x;
    if (k >= lanes || t >= pip_steps(maxlen)) return;
    const bool first = t == 0;
    const uint32_t total = off[nb - 1] + pad[nb - 1];
    const uint32_t groups = total >> 2;   // lists are padded to x4
    // the octet path needs 8 lanes per group: every launch has lanes >= nb (pip_buckets), and the
    // grid-uniform test below keeps 8 groups' lanes within this launch's lanes
    const size_t oct_max = nb / 8 < 16384 ? nb / 8 : 16384;
    if (groups <= oct_max && 8 * (size_t)groups <= lanes) {
        const uint32_t pos = (uint32_t)(4 * (k >> 3));
        if (pos >= total) return;   // whole octets leave together
        const uint32_t b = bid[pos];
        const uint32_t j = pos - off[b], L = len[b];
        if (t == tail_t && L > 4) return;   // k_pip_tail's list (whole octets leave together)
        const uint32_t r = L - j < 4 ? L - j : 4;
        const size_t base = first ? (size_t)start[b] + j : (size_t)off[b] + j;
        auto load = [&](uint32_t e) -> ge {
            if (!first) return Qin[base + e];
            if (keys32) return P[keys32[base + e] & imask];
            const uint32_t g = vals[base + e];
            return P[g - fdiv(g, fn) * fn.d];
        };
        const uint32_t e0 = (threadIdx.x & 4) ? 2u : 0u;   // quad A: elements 0, 1; quad B: 2, 3
        const bool has0 = e0 < r, has1 = e0 + 1 < r;
        const ge u = load(has0 ? e0 : 0u);
        const ge v = has1 ? load(e0 + 1) : u;
        ge sum = ge_op_quad<false>(u, v);   // computed on every quad; kept where the pair exists
        if (!has1) sum = u;
        const ge sB = ge_row_move<0x104>(sum);   // quad A takes quad B's sum
        ge y = ge_op_quad<false>(sum, sB);
        if (r <= 2) y = sum;
        if ((threadIdx.x & 7) == 0) {
            const bool fin = L <= 4;
            const uint32_t o = fin ? 0u : off2[b] + j / 4;
            *(fin ? &S[b] : &Qout[o]) = y;
            if (!fin) bid2[o] = b;
        }
        return;
    }
    const uint32_t pos = (uint32_t)(4 * k);
    if (pos >= total) return;
    const uint32_t b = bid[pos];
    const uint32_t j = pos - off[b], L = len[b];
    if (t == tail_t && L > 4) return;   // k_pip_tail's list
    const uint32_t r = L - j < 4 ? L - j : 4;
    const size_t base = first ? (size_t)start[b] + j : (size_t)off[b] + j;
    auto load = [&](uint32_t t) -> ge {
        if (!first) return Qin[base + t];
        if (keys32) return P[keys32[base + t] & imask];
        const uint32_t g = vals[base + t];
        return P[g - fdiv(g, fn) * fn.d];
    };
    // the first level adds two input points: when every active lane's second one has Z exactly 1
    // (affine inputs, a wave-uniform test), Z1 Z2 is fe_mul_one(Z1) — same bits, no product
    auto add_in = [&](const ge& a, const ge& b) -> ge {
        const geq q = ge_prep(b);
        return ge_add_qp<false>(a, &q, first && __all(fe_is_one(b.Z)));
    };
    ge y0 = load(0);
    if (r > 1) y0 = add_in(y0, load(1));
    if (r > 2) {
        ge y1 = load(2);
        if (r > 3) y1 = add_in(y1, load(3));
        y0 = ge_add(y0, y1);
    }
    // a group that is the whole list holds the bucket's sum (the bucket leaves the next layout)
    const bool fin = L <= 4;
    const uint32_t o = fin ? 0u : off2[b] + j / 4;
    *(fin ? &S[b] : &Qout[o]) = y0;
    if (!fin) bid2[o] = b;
}


// The bucket trees' last levels, staged in LDS.  From layer TAIL_LAYER on only a few lists are
// longer than 4 (the top window's deep buckets and the rare crowded ones), and the step launches
// past it are latency-bound (a few thousand busy lanes, one launch per two levels).  Step
// TAIL_LAYER still finishes the lists of 2..4 nodes (most of the lower windows' buckets of
// 257..1024 points, tens of thousands of them: one add per lane); every longer list gets a block
// here instead: it loads an aligned chunk of up to TAIL_CHUNK nodes of the list into
// LDS and runs the pairwise tree over it level by level, one pair per lane quad (ge_op_quad, the
// same products as ge_add), with a barrier per level; a list longer than a chunk leaves one root
// per chunk in place and goes round again.  Chunks are aligned to 512 = 2^9 list positions, so every
// node is the canonical tree's (the layer-TAIL_LAYER nodes are its level-2 TAIL_LAYER nodes): the same
// bits as the global steps.
constexpr int TAIL_LAYER = 4;
constexpr int TAIL_CHUNK = 512;
// HIPBP_PIP_TAIL_LAYER=t (1 .. 8; A/B runs): the LDS tail from layer t instead (t = 1: nearly every
// bucket summed in LDS by one block, the whole-bucket staging; same bits, the chunks stay aligned)
static int pip_tail_layer() {
    const char* e = getenv("HIPBP_PIP_TAIL_LAYER");
    const int t = e ? atoi(e) : TAIL_LAYER;
    return t < 1 ? 1 : t > 8 ? 8 : t;
}
__global__ __launch_bounds__(PTPB) void k_pip_tail(const uint32_t* __restrict__ tailq, const unsigned* __restrict__ tailn,
                                                  ge* Q, const uint32_t* __restrict__ off,
                                                  const uint32_t* __restrict__ len, ge* S) {
    __shared__ ge sh[TAIL_CHUNK];
    const int t = threadIdx.x;
    const unsigned nq = *tailn;
    for (unsigned qi = blockIdx.x; qi < nq; qi += gridDim.x) {   // block-uniform loop
        const uint32_t b = tailq[qi];
        ge* base = Q + off[b];
        uint32_t L = len[b];
        while (L > 1) {
            const uint32_t nch = (L + TAIL_CHUNK - 1) / TAIL_CHUNK;
            for (uint32_t c = 0; c < nch; c++) {
                const int cnt = (int)(L - c * TAIL_CHUNK < (uint32_t)TAIL_CHUNK ? L - c * TAIL_CHUNK : TAIL_CHUNK);
                for (int i = t; i < cnt; i += PTPB) sh[i] = base[(size_t)c * TAIL_CHUNK + i];
                __syncthreads();
                for (int st = 1; st < cnt; st <<= 1) {
                    const int pairs = (cnt - st + 2 * st - 1) / (2 * st);   // i = 2 st a with i + st < cnt
                    for (int a0 = 0; a0 < pairs; a0 += PTPB / 4) {         // block-uniform trip count
                        const int a = a0 + (t >> 2);
                        if (a < pairs) {   // pairs of one level touch disjoint entries
                            const ge r = ge_op_quad<false>(sh[2 * st * a], sh[2 * st * a + st]);
                            if ((t & 3) == 0) sh[2 * st * a] = r;
                        }
                        __syncthreads();
                    }
                }
                // chunk c's root to list position c: chunk 0 (positions 0 .. 511, c < 512) is already read
                if (t == 0) base[c] = sh[0];
                __syncthreads();
            }
            L = nch;
        }
        if (t == 0) S[b] = base[0];
        __syncthreads();
    }
}

// one block per (virtual) window v = m Wp + lw: pairwise tree over its NC <= PTPB chunk values, in
// LDS, into Sw[m W + w0 + lw] (MSM m's window sums, absolute window index).  A latency-bound
// chain of log2(NC) levels, so each add runs on a lane quad (ge_op_quad: the same products as
// ge_add, 3 product latencies instead of 9); quad a of a level forms the pair a of that level.
__global__ __launch_bounds__(PTPB) void k_pip_window(const ge* __restrict__ V, int NC, int Wp, int W, int w0, ge* Sw) {
    __shared__ ge sh[PTPB];
    const int t = threadIdx.x;
    if (t < NC) sh[t] = V[(size_t)blockIdx.x * NC + t];
    __syncthreads();
    for (int st = 1; st < NC; st <<= 1) {
        const int pairs = (NC - st + 2 * st - 1) / (2 * st);   // i = 2 st a with i + st < NC
        for (int a0 = 0; a0 < pairs; a0 += PTPB / 4) {         // block-uniform trip count
            const int a = a0 + (t >> 2);
            if (a < pairs) {   // pairs of one level touch disjoint entries
                const ge r = ge_op_quad<false>(sh[2 * st * a], sh[2 * st * a + st]);
                if ((t & 3) == 0) sh[2 * st * a] = r;
            }
            __syncthreads();
        }
    }
    if (t == 0) Sw[(size_t)(blockIdx.x / Wp) * W + w0 + blockIdx.x % Wp] = sh[0];
}

// ---- latency-bound chains: one point operation per lane QUAD (ge25519_quad.h).

// ---- the Horner chain: one point operation per 16-lane row, one product per lane quad.
// (fe_mul_q4, the product split over a lane quad: ge25519_quad.h)
// (fe_row_bcast: lane SRC of each 16-lane row to the whole row, ge25519_quad.h)
// DBL: add(p, p) (q ignored); else add(p, q).  p, q replicated over the row; result replicated.
// Quad qi of the row forms product qi of each stage (A, B, T1 T2, Z1 Z2 / X3, Y3, Z3, T3).
template <bool DBL>
__device__ __forceinline__ ge ge_op16(const ge& p, const ge& q) {
    const int qi = (threadIdx.x >> 2) & 3;
    const fe ymx = fe_sub(p.Y, p.X), ypx = fe_add(p.Y, p.X);
    const fe x1 = fe_sel4(qi, ymx, ypx, p.T, p.Z);
    fe r1;
    if (DBL) {
        r1 = fe_mul_q4(x1, x1);   // the squares: mul(f, f) == fe25519_sq's product
    } else {
        const fe qymx = fe_sub(q.Y, q.X), qypx = fe_add(q.Y, q.X);
        r1 = fe_mul_q4(x1, fe_sel4(qi, qymx, qypx, q.T, q.Z));
    }
    const fe A = fe_row_bcast<0>(r1), B = fe_row_bcast<4>(r1), CT = fe_row_bcast<8>(r1);
    fe D = fe_row_bcast<12>(r1);
    const fe C = fe_quad_bcast<0>(fe_mul_q4_k(CT));
    D = fe_add(D, D);
    const fe E = fe_sub(B, A), F = fe_sub(D, C), G = fe_add(D, C), H = fe_add(B, A);
    const fe r3 = fe_mul_q4(fe_sel4(qi, E, G, F, E), fe_sel4(qi, F, H, G, H));
    return ge{fe_row_bcast<0>(r3), fe_row_bcast<4>(r3), fe_row_bcast<8>(r3), fe_row_bcast<12>(r3)};
}

#ifndef BP_HORNER16   // 3: rows in operand form (default, r04j: one MSM 2.26/2.30 vs 2.33/2.34 ms with 1)
#define BP_HORNER16 3
#endif
// Horner over windows w_top .. w_end (descending): T = Tin ? *Tin : S_{w_top} (then from
// w_top - 1); per window c doublings, then + S_w.  A block (one wave) per MSM of the batch; each
// 16-lane row of the wave runs the chain (BP_HORNER16=3: the operand-form row step of sm_row;
// 1: ge_op16, a product per lane quad on replicated points; 2: operand-form quads; 0: ge_op_quad,
// 16 identical quads); lane 0 stores.  Split at any window, two calls give the single chain's bits.
__global__ __launch_bounds__(64) void k_pip_horner(const ge* __restrict__ Sw, int W, int w_top, int w_end, int c,
                                                  const ge* __restrict__ Tin, ge* out) {
    Sw += (size_t)blockIdx.x * W;   // block m: MSM m of the batch
    out += blockIdx.x;
    ge T;
    int w = w_top;
    if (Tin) {
        T = Tin[blockIdx.x];
    } else {
        T = Sw[w_top];
        w--;
    }
    if (BP_HORNER16 == 3) {   // 16-lane rows in operand form (ge25519_quad.h sm_row's step), 4 identical rows
        fe o = row_of_form(T), r3;
        bool pend = false;       // r3 holds the last operation's stage-3 products, o is stale
        for (; w >= w_end; w--) {
            for (int d = 0; d < c; d++) {
                if (pend) o = row_of_next(r3);
                r3 = ge_row_of_step(o, o);
                pend = true;
            }
            if (pend) o = row_of_next(r3);
            r3 = ge_row_of_step(o, row_of_form(Sw[w]));
            pend = true;
        }
        if (pend) T = row_of_point(r3);
    } else if (BP_HORNER16 == 2) {   // lane quads in operand form (ge25519_quad.h), squares for the doublings
        fe o = quad_of_form(T), r3;
        bool pend = false;       // r3 holds the last operation's stage-3 products, o is stale
        for (; w >= w_end; w--) {
            for (int d = 0; d < c; d++) {
                if (pend) o = quad_of_next(r3);
                r3 = ge_quad_of_step<true>(o, o);
                pend = true;
            }
            if (pend) o = quad_of_next(r3);
            r3 = ge_quad_of_step(o, quad_of_form(Sw[w]));
            pend = true;
        }
        if (pend) T = quad_of_point(r3);
    } else {
        for (; w >= w_end; w--) {
            if (BP_HORNER16) {
                for (int d = 0; d < c; d++) T = ge_op16<true>(T, T);
                T = ge_op16<false>(T, Sw[w]);
            } else {
                for (int d = 0; d < c; d++) T = ge_op_quad<true>(T, T);
                T = ge_op_quad<false>(T, Sw[w]);
            }
        }
    }
    if (threadIdx.x == 0) *out = T;
}

// chunk k of window w (one lane octet = two quads): buckets kM .. kM+M-1 -> V = S + (kM) R
// (orc_msm_pippenger).  The running sums R = R + B_j, S = S + R are two chains: quad A walks R,
// quad B walks S one step behind, fed each new R over DPP — both quads run the same point add in
// lockstep on their own operands, 15 dependent adds instead of 29.  (kM) R is
// ge25519_scalarmult's double-and-add on the scalar's raw bits, leading zeros from dtab.
__global__ __launch_bounds__(PTPB) void k_pip_chunks(const ge* __restrict__ Sb, int c, int W, ge* V,
                                                    const ge* __restrict__ dtab) {
    // Sb[b]: every bucket's sum (written by the step that finished it; empty buckets: ge25519_0)
    const size_t NB = (size_t)1 << c, NC = NB / PM;
    const size_t g = ((size_t)blockIdx.x * PTPB + threadIdx.x) >> 3;
    if (g >= (size_t)W * NC) return;   // whole octets leave together
    const bool qB = (threadIdx.x & 4) != 0;
    const size_t w = g / NC, k = g % NC, b0 = w * NB + k * PM;
    ge X = Sb[b0 + PM - 1];   // A: R = B_{M-1}; B: S = B_{M-1}
    ge Rin = X;
    for (int j = PM - 2; j >= 0; j--) {
        // A: R_j = R_{j+1} + B_j (j = 0: the final R + B_0);  B: S = S + R_{j+1} (from j = M-3 on)
        const ge y = qB ? Rin : Sb[b0 + j];
        const ge res = ge_op_quad<false>(X, y);
        if (!qB || j < PM - 2) X = res;
        Rin = ge_row_move<0x114>(X);   // quad B takes quad A's new R
    }
    // A holds R, B holds S
    const uint64_t km = (uint64_t)k * PM;
    ge r = dtab[km ? 192 + __clzll(km) : 256];
    if (km)
        for (int i = 63 - __clzll(km); i >= 0; i--) {
            r = ge_op_quad<true>(r, r);
            if ((km >> i) & 1) r = ge_op_quad<false>(r, X);
        }
    const ge S = ge_row_move<0x104>(X);   // quad A takes quad B's S
    r = ge_op_quad<false>(S, r);
    if ((threadIdx.x & 7) == 0) V[g] = r;
}

struct DBuf {
    void* p = nullptr;
    size_t cap = 0;
    hipError_t need(size_t bytes) {
        if (bytes <= cap) return hipSuccess;
        if (p) {   // growing: earlier MSMs on this workspace's streams may still read the old buffer
            hipError_t e = hipDeviceSynchronize();
            if (e == hipSuccess) e = hipFree(p);
            if (e != hipSuccess) return e;
            p = nullptr;
            cap = 0;
        }
        hipError_t e = hipMalloc(&p, bytes ? bytes : 1);
        if (e == hipSuccess) cap = bytes;
        return e;
    }
    template <typename T> T* as() const { return (T*)p; }
};
struct PipWs {
    DBuf keys_in, keys, vals, temp, start, len[2], lay, bq, bid[2], Q[2], S, V, Sw, Tmid, maxlen, part, tailq;
    hipStream_t side = nullptr;           // the Horner chain's stream
    hipEvent_t ev[4] = {};   // [1] top half's buckets done, [2] bottom half done, [3] chain done
};
// Workspaces per (device, stream): torch's default stream is handle 0 on every device, so the
// stream alone does not identify a workspace.  Each pair holds the top and bottom part's
// workspaces.  g_pip_mu guards the map (engines of different devices hold different locks);
// a workspace itself is used only under its device's engine lock.
struct PipPair { PipWs hi, lo; };
std::map<std::pair<int, hipStream_t>, PipPair*> g_pip;
std::mutex g_pip_mu;

inline unsigned nb_of(size_t items) { return (unsigned)((items + PTPB - 1) / PTPB); }
}  // namespace

#define PIP_RET(x) do { hipError_t _e = (x); if (_e != hipSuccess) return _e; } while (0)

// stable sort of the 16-bit digit keys on their low `bits` bits, values = 0, 1, 2, ... (rocPRIM
// onesweep with a counting iterator: 2 passes for 12 bits, no value array read)
static hipError_t pip_sort(void* temp, size_t& tb, const uint16_t* kin, uint16_t* kout, uint32_t* vout, size_t N,
                           int bits, hipStream_t s) {
    return rocprim::radix_sort_pairs(temp, tb, kin, kout, rocprim::counting_iterator<uint32_t>(0u), vout,
                                     (unsigned)N, 0u, (unsigned)bits, s);
}
// stable sort of the 32-bit keys (digit << ib | i) on bits [ib, ib + c): keys only
#ifdef BP_PIP_SORT_IPT   // A/B builds: onesweep tile (items per thread) and radix bits per pass
using PipSortCfg = rocprim::radix_sort_config<
    rocprim::default_config, rocprim::default_config,
    rocprim::radix_sort_onesweep_config<rocprim::kernel_config<1024, BP_PIP_SORT_IPT>,
                                        rocprim::kernel_config<1024, BP_PIP_SORT_IPT>, BP_PIP_SORT_BITS,
                                        rocprim::block_radix_rank_algorithm::match>>;
#else
using PipSortCfg = rocprim::default_config;
#endif
static hipError_t pip_sort32(void* temp, size_t& tb, const uint32_t* kin, uint32_t* kout, size_t N, int ib, int c,
                             hipStream_t s) {
    return rocprim::radix_sort_keys<PipSortCfg>(temp, tb, kin, kout, (unsigned)N, (unsigned)ib, (unsigned)(ib + c), s);
}
// HIPBP_PIP_KEYS16=1 forces the 16-bit-key path (read per call: tests run both paths in one process)
static bool pip_force16() {
    const char* e = getenv("HIPBP_PIP_KEYS16");
    return e && e[0] == '1';
}

// Bucket sums of windows [w0, w1) on stream s, into ws.S (the step that finishes a list writes it).
static hipError_t pip_buckets(PipWs& ws, const fe* scal, const ge* P, size_t n, size_t count, int c, int w0, int w1,
                              hipStream_t s) {
    const int Wp = w1 - w0;
    const size_t W = (size_t)Wp * count;   // virtual windows: the part's windows of every MSM
    const size_t NB = (size_t)1 << c, nb = W * NB, N = W * n, NC = NB / PM;
    int ib = 0;   // bits of the point index in a 32-bit key
    while (ib < 32 && ((size_t)1 << ib) < n) ib++;
    const bool k32 = c + ib <= 32 && !pip_force16();
    PIP_RET(ws.keys_in.need(N * (k32 ? 4 : 2)));
    PIP_RET(ws.keys.need(N * (k32 ? 4 : 2)));
    if (!k32) PIP_RET(ws.vals.need(N * 4));
    PIP_RET(ws.start.need(nb * 4));
    for (int i = 0; i < 2; i++) {
        PIP_RET(ws.len[i].need(nb * 4));
    }
    // the worst-case step count (a bucket list is at most n long); steps past the depth of the
    // data exit on the device (pip_steps), so nothing here waits for the GPU
    int levels = 1;
    while (levels < 31 && ((size_t)1 << levels) < n) levels++;
    const int steps = (levels + 1) / 2, T = steps + 1;   // layouts 0 .. steps, then the start layer T
    const unsigned nparts = (unsigned)((nb + SCAN_BLK - 1) / SCAN_BLK);
    PIP_RET(ws.lay.need((size_t)3 * (T + 1) * nb * 4));
    PIP_RET(ws.part.need((size_t)(T + 1) * nparts * 4));
    uint32_t* LEN = ws.lay.as<uint32_t>();
    uint32_t* PAD = LEN + (size_t)(T + 1) * nb;
    uint32_t* OFF = PAD + (size_t)(T + 1) * nb;
    // step 0 reads <= N + 3 nb padded positions and writes a quarter of them (+ padding)
    const size_t tot0 = N + 3 * nb, qcap = tot0 / 4 + 4 * nb;
    PIP_RET(ws.bid[0].need(tot0 * 4)); PIP_RET(ws.bid[1].need(qcap * 4));
    PIP_RET(ws.Q[0].need(qcap * sizeof(ge))); PIP_RET(ws.Q[1].need(qcap * sizeof(ge)));
    PIP_RET(ws.V.need((size_t)W * NC * sizeof(ge)));
    PIP_RET(ws.S.need(nb * sizeof(ge)));
    PIP_RET(ws.maxlen.need(3 * sizeof(unsigned)));
    const int TL = pip_tail_layer();
    const int TT = steps > TL ? TL : 0;   // the LDS tail takes over at layer TT (0: none)
    if (TT) PIP_RET(ws.tailq.need(nb * sizeof(uint32_t)));
    const size_t nbq = N / BID_PIECE + 1;   // bidfill queue capacity (further pieces of long lists)
    PIP_RET(ws.bq.need(nbq * sizeof(uint2)));
    size_t tb_sort = 0;
    if (k32)
        PIP_RET(pip_sort32(nullptr, tb_sort, ws.keys_in.as<uint32_t>(), ws.keys.as<uint32_t>(), N, ib, c, s));
    else
        PIP_RET(pip_sort(nullptr, tb_sort, ws.keys_in.as<uint16_t>(), ws.keys.as<uint16_t>(), ws.vals.as<uint32_t>(),
                         N, c, s));
    PIP_RET(ws.temp.need(tb_sort));

    const FastDiv fn = fastdiv_make((uint32_t)n);
    // keys_in rows start 8-byte (16-byte) aligned when n % 4 == 0 (DBuf memory)
    const bool v4 = n % 4 == 0;
    const unsigned kgrid = nb_of(v4 ? count * n / 4 : count * n);
    if (k32 && v4)
        k_pip_keys<4, uint32_t><<<kgrid, PTPB, 0, s>>>(scal, fn, (uint32_t)count, c, ib, w0, Wp, ws.keys_in.as<uint32_t>(),
                                                        ws.len[0].as<uint32_t>(), nb, ws.maxlen.as<unsigned>());
    else if (k32)
        k_pip_keys<1, uint32_t><<<kgrid, PTPB, 0, s>>>(scal, fn, (uint32_t)count, c, ib, w0, Wp, ws.keys_in.as<uint32_t>(),
                                                        ws.len[0].as<uint32_t>(), nb, ws.maxlen.as<unsigned>());
    else if (v4)
        k_pip_keys<4, uint16_t><<<kgrid, PTPB, 0, s>>>(scal, fn, (uint32_t)count, c, 0, w0, Wp, ws.keys_in.as<uint16_t>(),
                                                        ws.len[0].as<uint32_t>(), nb, ws.maxlen.as<unsigned>());
    else
        k_pip_keys<1, uint16_t><<<kgrid, PTPB, 0, s>>>(scal, fn, (uint32_t)count, c, 0, w0, Wp, ws.keys_in.as<uint16_t>(),
                                                        ws.len[0].as<uint32_t>(), nb, ws.maxlen.as<unsigned>());
    const uint32_t tpw = (uint32_t)((n + HIST_TILE - 1) / HIST_TILE);
    if (k32)
        k_pip_hist<uint32_t><<<(unsigned)(W * tpw), HIST_TPB, NB * 4, s>>>(ws.keys_in.as<uint32_t>(), (uint32_t)n, c,
                                                                           ib, tpw, ws.len[0].as<uint32_t>());
    else
        k_pip_hist<uint16_t><<<(unsigned)(W * tpw), HIST_TPB, NB * 4, s>>>(ws.keys_in.as<uint16_t>(), (uint32_t)n, c,
                                                                           0, tpw, ws.len[0].as<uint32_t>());
    // the counts in sorted order (transposed), for the start layer
    k_pip_len0<<<nb_of(nb), PTPB, 0, s>>>(ws.len[0].as<uint32_t>(), ws.len[1].as<uint32_t>(), nb, c, (uint32_t)W,
                                          ws.maxlen.as<unsigned>(), ws.S.as<ge>(), ws.bq.as<uint2>());
    // every step's layout (LEN, PAD, OFF)[t], t = 0 .. steps, and OFF[T] = the sorted-order starts
    k_pip_lay_part<<<dim3(nparts, T + 1), PTPB, 0, s>>>(ws.len[0].as<uint32_t>(), ws.len[1].as<uint32_t>(), T, nb,
                                                        LEN, PAD, ws.part.as<uint32_t>(), nparts, TT,
                                                        ws.tailq.as<uint32_t>(), ws.maxlen.as<unsigned>() + 2);
    k_pip_lay_fin<<<dim3(nparts, T + 1), PTPB, 0, s>>>(PAD, ws.part.as<uint32_t>(), nparts, nb, OFF);
    k_pip_start<<<nb_of(nb), PTPB, 0, s>>>(OFF + (size_t)T * nb, nb, c, (uint32_t)W, ws.start.as<uint32_t>());
    if (k32) {
        PIP_RET(pip_sort32(ws.temp.p, tb_sort, ws.keys_in.as<uint32_t>(), ws.keys.as<uint32_t>(), N, ib, c, s));
        k_pip_bidfill<<<nb_of((nb + nbq) * 64), PTPB, 0, s>>>(LEN, OFF, nb, ws.maxlen.as<unsigned>(),
                                                               ws.bq.as<uint2>(), ws.bid[0].as<uint32_t>());
    } else {
        PIP_RET(pip_sort(ws.temp.p, tb_sort, ws.keys_in.as<uint16_t>(), ws.keys.as<uint16_t>(), ws.vals.as<uint32_t>(),
                         N, c, s));
        k_pip_bid0<<<nb_of(N), PTPB, 0, s>>>(ws.keys.as<uint16_t>(), ws.vals.as<uint32_t>(), N, fn, c,
                                             ws.start.as<uint32_t>(), OFF, ws.bid[0].as<uint32_t>());
    }
    const uint32_t* keys32 = k32 ? ws.keys.as<uint32_t>() : nullptr;
    const uint32_t imask = ib >= 32 ? 0xFFFFFFFFu : (uint32_t)((1ull << ib) - 1);
    // step t: layout t -> t + 1, (bid, data)[t & 1] -> [(t + 1) & 1]
    // at least nb lanes in every step (step 0 too: when n < 2^c / 4 the padded total is below
    // 4 nb), so the octet tail path, which takes up to nb / 8 groups, always has its 8 lanes each
    size_t lanes = std::max((tot0 + 3) / 4, nb);
    for (int t = 0; t < (TT ? TT + 1 : steps); t++) {
        const int a = t & 1, b = a ^ 1;
        const size_t l0 = (size_t)t * nb, l1 = l0 + nb;
        k_pip_step<<<nb_of(lanes), PTPB, 0, s>>>(t, ws.maxlen.as<unsigned>(), P, fn, keys32, imask,
                                                  ws.vals.as<uint32_t>(),
                                                  ws.start.as<uint32_t>(), ws.Q[a].as<ge>(), ws.bid[a].as<uint32_t>(),
                                                  OFF + l0, LEN + l0, PAD + l0, OFF + l1, ws.Q[b].as<ge>(),
                                                  ws.bid[b].as<uint32_t>(), ws.S.as<ge>(), nb, lanes, TT ? TT : -1);
        lanes = lanes / 4 + nb;
    }
    if (TT)   // layer TT's lists that need more than one more step (written by step TT - 1 into Q[TT & 1]), in LDS
        k_pip_tail<<<(unsigned)std::min(nb, (size_t)2048), PTPB, 0, s>>>(
            ws.tailq.as<uint32_t>(), ws.maxlen.as<unsigned>() + 2, ws.Q[TT & 1].as<ge>(), OFF + (size_t)TT * nb,
            LEN + (size_t)TT * nb, ws.S.as<ge>());
    return hipGetLastError();
}

// Chunks -> window sums of windows [w0, w1) into Sw[w0 .. w1-1], on stream s (latency-bound).
static hipError_t pip_finish(PipWs& ws, size_t count, int c, int Wtot, int w0, int w1, ge* Sw, const ge* dtab,
                             hipStream_t s) {
    const int Wp = w1 - w0, W = Wp * (int)count;
    const size_t NC = ((size_t)1 << c) / PM;
    k_pip_chunks<<<nb_of(8 * (size_t)W * NC), PTPB, 0, s>>>(ws.S.as<ge>(), c, W, ws.V.as<ge>(), dtab);
    k_pip_window<<<W, PTPB, 0, s>>>(ws.V.as<ge>(), (int)NC, Wp, Wtot, w0, Sw);
    return hipGetLastError();
}

// The windows run as two halves, top half first, each with its own workspace.  The caller's
// stream carries the throughput work (sort + bucket trees of both halves, then the bottom half's
// chunks); a side stream carries the latency-bound chains: the top half's chunks + window trees
// + its part of the Horner chain (~126 dependent doublings) overlap the bottom half's bucket
// trees, and only the bottom half's chunks and Horner part remain at the end.  Same values,
// same bits.
static hipError_t pip_pair(PipPair** out, hipStream_t s) {
    int dev = 0;
    PIP_RET(hipGetDevice(&dev));
    std::lock_guard<std::mutex> lk(g_pip_mu);
    auto key = std::make_pair(dev, s);
    auto it = g_pip.find(key);
    if (it != g_pip.end()) { *out = it->second; return hipSuccess; }
    PipPair* pp = new PipPair();
    auto fail = [&](hipError_t e) {   // a half-made pair is never cached
        if (pp->hi.side) (void)hipStreamDestroy(pp->hi.side);
        for (auto& ev : pp->hi.ev)
            if (ev) (void)hipEventDestroy(ev);
        delete pp;
        return e;
    };
    hipError_t e;
    // a high-priority stream: HIP spreads streams over a few hardware queues, and one that
    // shared the caller's queue would serialize the chains behind the bottom half again
    int lo_pr = 0, hi_pr = 0;
    if ((e = hipDeviceGetStreamPriorityRange(&lo_pr, &hi_pr)) != hipSuccess) return fail(e);
    if ((e = hipStreamCreateWithPriority(&pp->hi.side, hipStreamNonBlocking, hi_pr)) != hipSuccess) return fail(e);
    for (auto& ev : pp->hi.ev)
        if ((e = hipEventCreateWithFlags(&ev, hipEventDisableTiming)) != hipSuccess) return fail(e);
    g_pip[key] = pp;
    *out = pp;
    return hipSuccess;
}

hipError_t msm_pippenger(ge* result, const fe* scal, const ge* P, size_t n, size_t count, int c, const ge* dtab,
                         hipStream_t s) {
    if (n == 0 || count == 0) return hipSuccess;
    PipPair* pp = nullptr;
    PIP_RET(pip_pair(&pp, s));
    PipWs& hi = pp->hi;
    PipWs& lo = pp->lo;
#ifndef BP_PIP_SPLIT8
#define BP_PIP_SPLIT8 3   // the bottom part's share of the windows, in eighths (3: measured best)
#endif
    const int W = (256 + c - 1) / c, wm = (W * BP_PIP_SPLIT8) / 8 > 0 ? (W * BP_PIP_SPLIT8) / 8 : 1;
    PIP_RET(hi.Sw.need(count * W * sizeof(ge)));
    PIP_RET(hi.Tmid.need(count * sizeof(ge)));
    ge* Sw = hi.Sw.as<ge>();
    PIP_RET(pip_buckets(hi, scal, P, n, count, c, wm, W, s));
    PIP_RET(hipEventRecord(hi.ev[1], s));
    PIP_RET(hipStreamWaitEvent(hi.side, hi.ev[1], 0));
    PIP_RET(pip_finish(hi, count, c, W, wm, W, Sw, dtab, hi.side));
    k_pip_horner<<<(unsigned)count, 64, 0, hi.side>>>(Sw, W, W - 1, wm, c, nullptr, hi.Tmid.as<ge>());
    PIP_RET(hipGetLastError());
    PIP_RET(pip_buckets(lo, scal, P, n, count, c, 0, wm, s));
    PIP_RET(pip_finish(lo, count, c, W, 0, wm, Sw, dtab, s));
    PIP_RET(hipEventRecord(hi.ev[2], s));
    PIP_RET(hipStreamWaitEvent(hi.side, hi.ev[2], 0));
    k_pip_horner<<<(unsigned)count, 64, 0, hi.side>>>(Sw, W, wm - 1, 0, c, hi.Tmid.as<ge>(), result);
    PIP_RET(hipGetLastError());
    PIP_RET(hipEventRecord(hi.ev[3], hi.side));
    PIP_RET(hipStreamWaitEvent(s, hi.ev[3], 0));          // the result is ready in the caller's stream order
    return hipSuccess;
}

// Window sums of windows [w0, w1) of one MSM into Sw[w0 .. w1) (entries outside untouched), all on
// stream s: the same keys, sort, bucket trees, chunks and window trees as msm_pippenger's parts,
// so each S_w has the bits the single call forms.  A multi-GPU MSM gives each rank a window range
// and exchanges the 128-byte sums (cudabulletproof_amd/shard.py sharded_msm_pippenger).
hipError_t msm_pippenger_windows(ge* Sw, const fe* scal, const ge* P, size_t n, int c, int w0, int w1,
                                 const ge* dtab, hipStream_t s) {
    const int W = (256 + c - 1) / c;
    if (n == 0 || w0 >= w1 || w0 < 0 || w1 > W) return hipSuccess;
    PipPair* pp = nullptr;
    PIP_RET(pip_pair(&pp, s));
    PIP_RET(pip_buckets(pp->lo, scal, P, n, 1, c, w0, w1, s));
    return pip_finish(pp->lo, 1, c, W, w0, w1, Sw, dtab, s);
}

// Frees stream s's workspace pair on the current device (hipbp_release_stream_workspaces): waits
// for s and the pair's side stream, frees every buffer, destroys the side stream and events.
hipError_t pippenger_release(hipStream_t s) {
    int dev = 0;
    PIP_RET(hipGetDevice(&dev));
    PipPair* pp = nullptr;
    {
        std::lock_guard<std::mutex> lk(g_pip_mu);
        auto it = g_pip.find(std::make_pair(dev, s));
        if (it == g_pip.end()) return hipSuccess;
        pp = it->second;
        g_pip.erase(it);
    }
    // keep freeing after an error (the pair is already out of the map): the first error is returned
    hipError_t first = hipStreamSynchronize(s);
    auto keep = [&first](hipError_t r) { if (first == hipSuccess) first = r; };
    if (pp->hi.side) keep(hipStreamSynchronize(pp->hi.side));
    for (PipWs* w : {&pp->hi, &pp->lo}) {
        for (DBuf* b : {&w->keys_in, &w->keys, &w->vals, &w->temp, &w->start, &w->len[0], &w->len[1], &w->lay,
                        &w->bq, &w->bid[0], &w->bid[1], &w->Q[0], &w->Q[1], &w->S, &w->V, &w->Sw, &w->Tmid,
                        &w->maxlen, &w->part, &w->tailq})
            if (b->p) {
                keep(hipFree(b->p));
                b->p = nullptr;
            }
        for (auto& ev : w->ev)
            if (ev) {
                keep(hipEventDestroy(ev));
                ev = nullptr;
            }
        if (w->side) {
            keep(hipStreamDestroy(w->side));
            w->side = nullptr;
        }
    }
    delete pp;
    return first;
}

// Horner over all W window sums of `count` MSMs (Sw[m W .. m W + W)), on stream s.
hipError_t pippenger_horner(ge* result, const ge* Sw, size_t count, int c, hipStream_t s) {
    if (count == 0) return hipSuccess;
    const int W = (256 + c - 1) / c;
    k_pip_horner<<<(unsigned)count, 64, 0, s>>>(Sw, W, W - 1, 0, c, nullptr, result);
    return hipGetLastError();
}

}  // namespace bp
