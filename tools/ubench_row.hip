// ubench_row.hip — latency of the 16-lane row form (ge25519_quad.h sm_row): one wave (four rows,
// four items) running whole 256-bit scalar multiplications alone on its SIMD, the regime of a
// one-proof call's ticks.  Prints cycles per point operation (clock64 inside the kernel) and
// checks every result against the per-lane form (scalarmult, the bits of ge25519_scalarmult).
// Built with the same -D options as the library to A/B a row-form variant:
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 [-D...] tools/ubench_row.hip -o tools/ubench_row
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <vector>

#include "../cudabulletproof_amd/csrc/ge25519_dev.h"
#include "../cudabulletproof_amd/csrc/ge25519_quad.h"

using namespace bp;

__global__ void k_dtab(ge* dtab) {   // dtab[i] = i doublings of the identity (the leading-zero starts)
    if (threadIdx.x != 0) return;
    ge r{{{0, 0, 0, 0}}, {{1, 0, 0, 0}}, {{1, 0, 0, 0}}, {{0, 0, 0, 0}}};
    for (int i = 0; i <= 256; i++) {
        dtab[i] = r;
        r = ge_dbl(r);
    }
}

__global__ void k_row(ge* out, const fe* s, const ge* P, const ge* dtab, unsigned long long* clk, int reps) {
    const int item = threadIdx.x >> 4;
    ge r;
    const unsigned long long t0 = clock64();
    for (int k = 0; k < reps; k++) r = sm_row(s[item + 4 * k], P[item], dtab, nullptr, 0);
    const unsigned long long t1 = clock64();
    if ((threadIdx.x & 15) == 0) out[item] = r;
    if (threadIdx.x == 0) *clk = t1 - t0;
}

__global__ void k_lane(ge* out, const fe* s, const ge* P, const ge* dtab, int reps) {
    __shared__ geq qs[64];
    if (threadIdx.x >= 4) return;
    ge r;
    for (int k = 0; k < reps; k++) r = scalarmult<false>(s[threadIdx.x + 4 * k], P[threadIdx.x], &qs[threadIdx.x], dtab);
    out[threadIdx.x] = r;
}

int main() {
    const int reps = 8;
    std::vector<fe> hs(4 * reps);
    std::vector<ge> hp(4);
    uint64_t x = 0x9E3779B97F4A7C15ull;
    auto nx = [&]() { x ^= x << 13; x ^= x >> 7; x ^= x << 17; return x; };
    int ops = 0;
    for (auto& f : hs) {
        for (int k = 0; k < 4; k++) f.v[k] = nx();
        f.v[3] |= 1ull << 63;   // full-length scalars: 255 doublings + one add per set bit
    }
    for (int it = 0; it < 4; it++) {   // the wave runs until its longest row's chain ends
        int n = 0;
        for (int k = 0; k < reps; k++)
            for (int b = 254; b >= 0; b--) n += 1 + (int)((hs[it + 4 * k].v[b >> 6] >> (b & 63)) & 1);
        ops = n > ops ? n : ops;
    }
    for (auto& g : hp) {
        uint64_t* w = (uint64_t*)&g;
        for (int k = 0; k < 16; k++) w[k] = nx() & (k % 4 == 3 ? 0x7FFFFFFFFFFFFFFFull : ~0ull);
    }
    fe* ds;
    ge *dp, *dtab, *o1, *o2;
    unsigned long long* dclk;
    (void)hipMalloc(&ds, hs.size() * sizeof(fe));
    (void)hipMalloc(&dp, 4 * sizeof(ge));
    (void)hipMalloc(&dtab, 257 * sizeof(ge));
    (void)hipMalloc(&o1, 4 * sizeof(ge));
    (void)hipMalloc(&o2, 4 * sizeof(ge));
    (void)hipMalloc(&dclk, 8);
    (void)hipMemcpy(ds, hs.data(), hs.size() * sizeof(fe), hipMemcpyHostToDevice);
    (void)hipMemcpy(dp, hp.data(), 4 * sizeof(ge), hipMemcpyHostToDevice);
    k_dtab<<<1, 64>>>(dtab);
    k_row<<<1, 64>>>(o1, ds, dp, dtab, dclk, reps);   // warm (code load)
    (void)hipDeviceSynchronize();
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0);
    k_row<<<1, 64>>>(o1, ds, dp, dtab, dclk, reps);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    k_lane<<<1, 64>>>(o2, ds, dp, dtab, reps);
    (void)hipDeviceSynchronize();
    unsigned long long c = 0;
    (void)hipMemcpy(&c, dclk, 8, hipMemcpyDeviceToHost);
    std::vector<ge> r1(4), r2(4);
    (void)hipMemcpy(r1.data(), o1, 4 * sizeof(ge), hipMemcpyDeviceToHost);
    (void)hipMemcpy(r2.data(), o2, 4 * sizeof(ge), hipMemcpyDeviceToHost);
    const bool match = memcmp(r1.data(), r2.data(), 4 * sizeof(ge)) == 0;
    printf("{\"ops\": %d, \"cycles_per_op\": %.1f, \"us_per_op\": %.3f, \"ms\": %.3f, \"match\": %s}\n", ops,
           (double)c / ops, ms * 1e3 / ops, ms, match ? "true" : "false");
    return match ? 0 : 1;
}
