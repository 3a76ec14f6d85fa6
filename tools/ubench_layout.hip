// ubench_layout.hip — A/B of the point layout in HBM, memory alone: 128-B AoS points (X|Y|Z|T,
// 4 u64 limbs each, what the library stores; a lane moves a point with 8 dwordx4) against limb-plane
// SoA (16 planes of u64, plane p holds limb p of every point; a lane moves a point with 16 dwordx2
// that are coalesced across the wave when the points are consecutive).  Two access patterns, the two
// the verify tick has:
//   gather — lane i reads point idx[i] of a 2^23-point (1 GiB) table at a random index and writes
//            point i of the output: the prefix-table entry a fixed-base scalar-mult starts from;
//   stream — lane i reads point i and writes point i: terms written by one tick, read by the next.
// Prints GB/s of the bytes the lanes ask for (128 read + 128 written per point, + 4 B of index for
// gather), per layout and pattern; the point counts are 2^22 per launch.
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <vector>

constexpr int LIMBS = 16;   // u64 per point
constexpr uint32_t TAB_LOG2 = 23, N_LOG2 = 22;

__global__ void __launch_bounds__(256) aos_gather(const uint4* __restrict__ tab, const uint32_t* __restrict__ idx,
                                                  uint4* __restrict__ out, uint32_t n) {
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const uint4* src = tab + (size_t)idx[i] * 8;
    uint4 v[8];
#pragma unroll
    for (int k = 0; k < 8; k++) v[k] = src[k];
#pragma unroll
    for (int k = 0; k < 8; k++) out[(size_t)i * 8 + k] = v[k];
}

__global__ void __launch_bounds__(256) soa_gather(const uint64_t* __restrict__ tab, const uint32_t* __restrict__ idx,
                                                  uint64_t* __restrict__ out, uint32_t n, uint32_t m) {
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const uint32_t j = idx[i];
    uint64_t v[LIMBS];
#pragma unroll
    for (int p = 0; p < LIMBS; p++) v[p] = tab[(size_t)p * m + j];
#pragma unroll
    for (int p = 0; p < LIMBS; p++) out[(size_t)p * n + i] = v[p];
}

__global__ void __launch_bounds__(256) aos_stream(const uint4* __restrict__ in, uint4* __restrict__ out, uint32_t n) {
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    uint4 v[8];
#pragma unroll
    for (int k = 0; k < 8; k++) v[k] = in[(size_t)i * 8 + k];
#pragma unroll
    for (int k = 0; k < 8; k++) out[(size_t)i * 8 + k] = v[k];
}

__global__ void __launch_bounds__(256) soa_stream(const uint64_t* __restrict__ in, uint64_t* __restrict__ out, uint32_t n) {
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    uint64_t v[LIMBS];
#pragma unroll
    for (int p = 0; p < LIMBS; p++) v[p] = in[(size_t)p * n + i];
#pragma unroll
    for (int p = 0; p < LIMBS; p++) out[(size_t)p * n + i] = v[p];
}

#define CK(x)                                                             \
    do {                                                                  \
        hipError_t e_ = (x);                                              \
        if (e_ != hipSuccess) {                                           \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));       \
            return 1;                                                     \
        }                                                                 \
    } while (0)

template <class F>
static float time_ms(F launch, int reps) {
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    launch();
    launch();
    (void)hipEventRecord(a);
    for (int r = 0; r < reps; r++) launch();
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, a, b);
    (void)hipEventDestroy(a);
    (void)hipEventDestroy(b);
    return ms / reps;
}

int main() {
    const uint32_t m = 1u << TAB_LOG2, n = 1u << N_LOG2;
    const size_t tab_bytes = (size_t)m * LIMBS * 8, pts_bytes = (size_t)n * LIMBS * 8;
    void *tab, *in, *out;
    uint32_t* idx;
    CK(hipMalloc(&tab, tab_bytes));
    CK(hipMalloc(&in, pts_bytes));
    CK(hipMalloc(&out, pts_bytes));
    CK(hipMalloc(&idx, (size_t)n * 4));
    CK(hipMemset(tab, 0x5a, tab_bytes));
    CK(hipMemset(in, 0xa5, pts_bytes));
    std::vector<uint32_t> h(n);
    uint64_t s = 0x9e3779b97f4a7c15ull;
    for (uint32_t i = 0; i < n; i++) {
        s ^= s << 13; s ^= s >> 7; s ^= s << 17;
        h[i] = (uint32_t)(s % m);
    }
    CK(hipMemcpy(idx, h.data(), (size_t)n * 4, hipMemcpyHostToDevice));
    const dim3 grid(n / 256), blk(256);
    const int reps = 20;
    const float g_aos = time_ms([&] { aos_gather<<<grid, blk>>>((const uint4*)tab, idx, (uint4*)out, n); }, reps);
    const float g_soa = time_ms([&] { soa_gather<<<grid, blk>>>((const uint64_t*)tab, idx, (uint64_t*)out, n, m); }, reps);
    const float s_aos = time_ms([&] { aos_stream<<<grid, blk>>>((const uint4*)in, (uint4*)out, n); }, reps);
    const float s_soa = time_ms([&] { soa_stream<<<grid, blk>>>((const uint64_t*)in, (uint64_t*)out, n); }, reps);
    CK(hipGetLastError());
    CK(hipDeviceSynchronize());
    const double gb_g = (double)n * (256 + 4) / 1e9, gb_s = (double)n * 256 / 1e9;
    printf("{\"points_per_launch\": %u, \"table_points\": %u, \"ms\": {\"gather_aos\": %.4f, \"gather_soa\": %.4f, "
           "\"stream_aos\": %.4f, \"stream_soa\": %.4f}, \"GBps\": {\"gather_aos\": %.1f, \"gather_soa\": %.1f, "
           "\"stream_aos\": %.1f, \"stream_soa\": %.1f}}\n",
           n, m, g_aos, g_soa, s_aos, s_soa, gb_g / (g_aos * 1e-3), gb_g / (g_soa * 1e-3), gb_s / (s_aos * 1e-3),
           gb_s / (s_soa * 1e-3));
    return 0;
}
