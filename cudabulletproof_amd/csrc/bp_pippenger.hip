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
// GPU mapping.  (1) one (key = w<<c | digit, value = i) pair per window and point, stable radix
// sort (hipCUB) -> each bucket's points contiguous in index order; bucket bounds from the sorted
// keys (no atomics).  (2) the bucket trees level by level over ALL buckets at once: a level's
// lane takes one adjacent pair of one bucket's current list (lists compacted and padded to even
// length after every level, offsets by an exclusive scan), so every lane of every wave adds —
// ~W n point additions at the VALU roof instead of one lane walking a bucket.  (3) one lane per
// chunk (W 2^c / 16 lanes) for the running sums and the small scalar-mult, (4) one block per
// window: the chunk tree in LDS, (5) one lane: the Horner chain (~256 doublings, latency-bound).
#include <hipcub/hipcub.hpp>

#include <map>
#include <mutex>

#include "bp_kernels.h"
#include "ge25519_dev.h"

namespace bp {

namespace {
constexpr int PTPB = 256;
constexpr int PM = 16;   // buckets per chunk

__global__ __launch_bounds__(PTPB) void k_pip_keys(const fe* __restrict__ s, size_t n, int c, int W,
                                                  uint32_t* keys, uint32_t* vals) {
    const size_t g = (size_t)blockIdx.x * PTPB + threadIdx.x;
    if (g >= (size_t)W * n) return;
    const int w = (int)(g / n);
    const size_t i = g % n;
    const int lo = c * w;
    // bits [lo, lo + c) of the 256-bit scalar (a window may straddle two limbs or end past bit 255)
    const fe sc = s[i];
    const int li = lo >> 6, sh = lo & 63;
    uint64_t v = sc.v[li] >> sh;
    if (sh && li < 3) v |= sc.v[li + 1] << (64 - sh);
    const uint32_t d = (uint32_t)(v & ((1ull << c) - 1));
    keys[g] = ((uint32_t)w << c) | d;
    vals[g] = (uint32_t)i;
}

// first/last occurrence of each key in the sorted array -> bucket start and length
__global__ __launch_bounds__(PTPB) void k_pip_bounds(const uint32_t* __restrict__ keys, size_t N,
                                                    uint32_t* start, uint32_t* len) {
    const size_t p = (size_t)blockIdx.x * PTPB + threadIdx.x;
    if (p >= N) return;
    const uint32_t k = keys[p];
    if (p == 0 || keys[p - 1] != k) start[k] = (uint32_t)p;
    if (p == N - 1 || keys[p + 1] != k) len[k] = (uint32_t)(p + 1);   // end, made a length below
}

__global__ __launch_bounds__(PTPB) void k_pip_len0(const uint32_t* __restrict__ start, uint32_t* len, uint32_t* pad,
                                                  size_t nb, unsigned* maxlen) {
    const size_t b = (size_t)blockIdx.x * PTPB + threadIdx.x;
    if (b >= nb) return;
    const uint32_t L = len[b] ? len[b] - start[b] : 0;
    len[b] = L;
    pad[b] = L + (L & 1);
    if (L) atomicMax(maxlen, L);
}

__global__ __launch_bounds__(PTPB) void k_pip_nextlen(const uint32_t* __restrict__ len, uint32_t* len2, uint32_t* pad2,
                                                     size_t nb) {
    const size_t b = (size_t)blockIdx.x * PTPB + threadIdx.x;
    if (b >= nb) return;
    const uint32_t L = (len[b] + 1) >> 1;
    len2[b] = L;
    pad2[b] = L + (L & 1);
}

// largest b with off[b] <= pos (zero-length buckets share the next bucket's offset, so this is
// the bucket whose padded region holds pos)
__device__ __forceinline__ size_t bucket_of(const uint32_t* __restrict__ off, size_t nb, uint32_t pos) {
    size_t lo = 0, hi = nb;   // invariant: off[lo] <= pos, answer in [lo, hi)
    while (hi - lo > 1) {
        size_t mid = (lo + hi) >> 1;
        if (off[mid] <= pos) lo = mid;
        else hi = mid;
    }
    return lo;
}

// One tree level over every bucket: lane k takes positions (2k, 2k+1) of the current padded
// layout; pairs add, an odd bucket's last element is carried.  Level 0 reads the points through
// the sorted indices.
__global__ __launch_bounds__(PTPB) void k_pip_level(int first, const ge* __restrict__ P,
                                                   const uint32_t* __restrict__ vals,
                                                   const uint32_t* __restrict__ start, const ge* __restrict__ Qin,
                                                   const uint32_t* __restrict__ off, const uint32_t* __restrict__ len,
                                                   const uint32_t* __restrict__ pad,
                                                   const uint32_t* __restrict__ off2, ge* Qout, size_t nb,
                                                   size_t lanes) {
    const size_t k = (size_t)blockIdx.x * PTPB + threadIdx.x;
    if (k >= lanes) return;
    const uint32_t total = off[nb - 1] + pad[nb - 1];
    const uint32_t pos = (uint32_t)(2 * k);
    if (pos >= total) return;
    const size_t b = bucket_of(off, nb, pos);
    const uint32_t j = pos - off[b], L = len[b];
    if (j >= L) return;   // padding
    ge x0, out;
    if (first) x0 = P[vals[start[b] + j]];
    else x0 = Qin[off[b] + j];
    if (j + 1 < L) {
        ge x1;
        if (first) x1 = P[vals[start[b] + j + 1]];
        else x1 = Qin[off[b] + j + 1];
        out = ge_add(x0, x1);
    } else {
        out = x0;
    }
    Qout[off2[b] + j / 2] = out;
}

__device__ __forceinline__ ge bucket_sum(const ge* __restrict__ Q, const uint32_t* __restrict__ off,
                                         const uint32_t* __restrict__ cnt, size_t b) {
    return cnt[b] ? Q[off[b]] : ge_zero();
}

// chunk k of window w: buckets kM .. kM+M-1 -> V = S + (kM) R (orc_msm_pippenger)
__global__ __launch_bounds__(PTPB) void k_pip_chunks(const ge* __restrict__ Q, const uint32_t* __restrict__ off,
                                                    const uint32_t* __restrict__ cnt, int c, int W, ge* V,
                                                    const ge* __restrict__ dtab) {
    __shared__ geq qs[PTPB];
    const size_t NB = (size_t)1 << c, NC = NB / PM;
    const size_t g = (size_t)blockIdx.x * PTPB + threadIdx.x;
    if (g >= (size_t)W * NC) return;
    const size_t w = g / NC, k = g % NC, b0 = w * NB + k * PM;
    ge R = bucket_sum(Q, off, cnt, b0 + PM - 1), S = R;
    for (int j = PM - 2; j >= 1; j--) {
        R = ge_add(R, bucket_sum(Q, off, cnt, b0 + j));
        S = ge_add(S, R);
    }
    R = ge_add(R, bucket_sum(Q, off, cnt, b0));
    fe km = fe_set((uint64_t)k * PM);
    ge sm = scalarmult<true>(km, R, &qs[threadIdx.x], dtab);
    V[g] = ge_add(S, sm);
}

// one block per window: pairwise tree over its NC <= PTPB chunk values, in LDS
__global__ __launch_bounds__(PTPB) void k_pip_window(const ge* __restrict__ V, int NC, ge* Sw) {
    __shared__ ge sh[PTPB];
    const int t = threadIdx.x;
    if (t < NC) sh[t] = V[(size_t)blockIdx.x * NC + t];
    __syncthreads();
    for (int st = 1; st < NC; st <<= 1) {
        if ((t % (2 * st)) == 0 && t + st < NC) sh[t] = ge_add(sh[t], sh[t + st]);
        __syncthreads();
    }
    if (t == 0) Sw[blockIdx.x] = sh[0];
}

__global__ void k_pip_horner(const ge* __restrict__ Sw, int W, int c, ge* out) {
    if (threadIdx.x != 0) return;
    ge T = Sw[W - 1];
    for (int w = W - 2; w >= 0; w--) {
        for (int d = 0; d < c; d++) T = ge_dbl(T);   // add(T, T): the same bits
        T = ge_add(T, Sw[w]);
    }
    *out = T;
}

struct DBuf {
    void* p = nullptr;
    size_t cap = 0;
    hipError_t need(size_t bytes) {
        if (bytes <= cap) return hipSuccess;
        if (p) { hipError_t e = hipFree(p); if (e != hipSuccess) return e; p = nullptr; cap = 0; }
        hipError_t e = hipMalloc(&p, bytes ? bytes : 1);
        if (e == hipSuccess) cap = bytes;
        return e;
    }
    template <typename T> T* as() const { return (T*)p; }
};
struct PipWs {
    DBuf keys_in, vals_in, keys, vals, temp, start, len[2], pad[2], off[2], Q[2], V, Sw, maxlen;
    unsigned* host_max = nullptr;
};
std::map<hipStream_t, PipWs*> g_pip;   // per stream; callers hold the engine lock

inline unsigned nb_of(size_t items) { return (unsigned)((items + PTPB - 1) / PTPB); }
}  // namespace

#define PIP_RET(x) do { hipError_t _e = (x); if (_e != hipSuccess) return _e; } while (0)

hipError_t msm_pippenger(ge* result, const fe* scal, const ge* P, size_t n, int c, const ge* dtab, hipStream_t s) {
    if (n == 0) return hipSuccess;
    PipWs*& wsp = g_pip[s];
    if (!wsp) {
        wsp = new PipWs();
        PIP_RET(hipHostMalloc(&wsp->host_max, sizeof(unsigned)));
    }
    PipWs& ws = *wsp;
    const int W = (256 + c - 1) / c;
    const size_t NB = (size_t)1 << c, nb = (size_t)W * NB, N = (size_t)W * n, NC = NB / PM;
    int kbits = c;
    while ((1 << (kbits - c)) < W) kbits++;
    PIP_RET(ws.keys_in.need(N * 4)); PIP_RET(ws.vals_in.need(N * 4));
    PIP_RET(ws.keys.need(N * 4)); PIP_RET(ws.vals.need(N * 4));
    PIP_RET(ws.start.need(nb * 4));
    for (int i = 0; i < 2; i++) {
        PIP_RET(ws.len[i].need(nb * 4)); PIP_RET(ws.pad[i].need(nb * 4)); PIP_RET(ws.off[i].need(nb * 4));
    }
    // level outputs: at most (N + nb) / 2 points after level 0, halving (plus padding) after
    const size_t qcap = (N + nb) / 2 + nb;
    PIP_RET(ws.Q[0].need(qcap * sizeof(ge))); PIP_RET(ws.Q[1].need(qcap * sizeof(ge)));
    PIP_RET(ws.V.need((size_t)W * NC * sizeof(ge))); PIP_RET(ws.Sw.need((size_t)W * sizeof(ge)));
    PIP_RET(ws.maxlen.need(sizeof(unsigned)));
    size_t tb_sort = 0, tb_scan = 0;
    PIP_RET(hipcub::DeviceRadixSort::SortPairs(nullptr, tb_sort, ws.keys_in.as<uint32_t>(), ws.keys.as<uint32_t>(),
                                               ws.vals_in.as<uint32_t>(), ws.vals.as<uint32_t>(), (int)N, 0, kbits, s));
    PIP_RET(hipcub::DeviceScan::ExclusiveSum(nullptr, tb_scan, ws.pad[0].as<uint32_t>(), ws.off[0].as<uint32_t>(),
                                             (int)nb, s));
    PIP_RET(ws.temp.need(tb_sort > tb_scan ? tb_sort : tb_scan));

    k_pip_keys<<<nb_of(N), PTPB, 0, s>>>(scal, n, c, W, ws.keys_in.as<uint32_t>(), ws.vals_in.as<uint32_t>());
    PIP_RET(hipcub::DeviceRadixSort::SortPairs(ws.temp.p, tb_sort, ws.keys_in.as<uint32_t>(), ws.keys.as<uint32_t>(),
                                               ws.vals_in.as<uint32_t>(), ws.vals.as<uint32_t>(), (int)N, 0, kbits, s));
    PIP_RET(hipMemsetAsync(ws.start.p, 0, nb * 4, s));
    PIP_RET(hipMemsetAsync(ws.len[0].p, 0, nb * 4, s));
    PIP_RET(hipMemsetAsync(ws.maxlen.p, 0, sizeof(unsigned), s));
    k_pip_bounds<<<nb_of(N), PTPB, 0, s>>>(ws.keys.as<uint32_t>(), N, ws.start.as<uint32_t>(), ws.len[0].as<uint32_t>());
    k_pip_len0<<<nb_of(nb), PTPB, 0, s>>>(ws.start.as<uint32_t>(), ws.len[0].as<uint32_t>(), ws.pad[0].as<uint32_t>(),
                                          nb, ws.maxlen.as<unsigned>());
    PIP_RET(hipcub::DeviceScan::ExclusiveSum(ws.temp.p, tb_scan, ws.pad[0].as<uint32_t>(), ws.off[0].as<uint32_t>(),
                                             (int)nb, s));
    PIP_RET(hipMemcpyAsync(ws.host_max, ws.maxlen.p, sizeof(unsigned), hipMemcpyDeviceToHost, s));
    PIP_RET(hipStreamSynchronize(s));
    int levels = 1;
    while (((size_t)1 << levels) < *ws.host_max) levels++;
    // level l: layout (off, len, pad)[l & 1] -> (.., ..)[(l + 1) & 1], data Q[(l + 1) & 1] (l >= 1 reads Q[l & 1])
    size_t lanes = (N + nb + 1) / 2;
    for (int l = 0; l < levels; l++) {
        const int a = l & 1, b = a ^ 1;
        k_pip_nextlen<<<nb_of(nb), PTPB, 0, s>>>(ws.len[a].as<uint32_t>(), ws.len[b].as<uint32_t>(),
                                                  ws.pad[b].as<uint32_t>(), nb);
        PIP_RET(hipcub::DeviceScan::ExclusiveSum(ws.temp.p, tb_scan, ws.pad[b].as<uint32_t>(),
                                                 ws.off[b].as<uint32_t>(), (int)nb, s));
        k_pip_level<<<nb_of(lanes), PTPB, 0, s>>>(l == 0, P, ws.vals.as<uint32_t>(), ws.start.as<uint32_t>(),
                                                   ws.Q[a].as<ge>(), ws.off[a].as<uint32_t>(),
                                                   ws.len[a].as<uint32_t>(), ws.pad[a].as<uint32_t>(),
                                                   ws.off[b].as<uint32_t>(), ws.Q[b].as<ge>(), nb, lanes);
        lanes = lanes / 2 + nb;
    }
    // after the last level every non-empty bucket holds its sum at off[levels & 1][b]
    const int fin = levels & 1;
    // a bucket is empty iff its level-0 length was 0 == its final length is 0
    k_pip_chunks<<<nb_of((size_t)W * NC), PTPB, 0, s>>>(ws.Q[fin].as<ge>(), ws.off[fin].as<uint32_t>(),
                                                         ws.len[fin].as<uint32_t>(), c, W, ws.V.as<ge>(), dtab);
    k_pip_window<<<W, PTPB, 0, s>>>(ws.V.as<ge>(), (int)NC, ws.Sw.as<ge>());
    k_pip_horner<<<1, 64, 0, s>>>(ws.Sw.as<ge>(), W, c, result);
    return hipGetLastError();
}

}  // namespace bp
