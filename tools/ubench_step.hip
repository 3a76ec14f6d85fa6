// ubench_step.hip — the VALU roof of the verify's own instruction mix: the point-operation loops
// of k_terms (ge25519_dev.h) run from registers and LDS only, no global memory inside the loop,
// at k_terms' occupancy (256-thread blocks, 4 per CU = 4 waves per SIMD, the q-side operands
// in LDS as k_terms keeps them), every SIMD busy for the whole run (one full round of blocks,
// no tail).  What it sustains in VALU wave-instructions per second is the peak the same mix can
// reach on this chip; k_terms' achieved rate (SQ_INSTS_VALU of the timed launches / their wall
// time, bench.py valu_roofline) divided by it is k_terms' fraction of that roof.
//   step   the per-lane unified step ge_add_sel<true, ZONE = true> (add(r, r) or add(r, P) per lane,
//          about one add in three as in a 255-bit scalar's chain)
//   dbl    the uniform loop's doubling ge_dbl
//   add    the uniform loop's add ge_add_qp<true> with Z2 = 1
// Prints one JSON object per variant: wall ms and the shader clock (clock64 / wall_clock64);
// the VALU instruction count comes from a rocprofv3 --pmc SQ_INSTS_VALU pass over the same
// binary (tools/valu_model.py combines them).
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <vector>

#include "../cudabulletproof_amd/csrc/ge25519_dev.h"

using namespace bp;

#define STEPS 768

template <int KIND>
__global__ __launch_bounds__(256, 4) void k_step(ge* out, const ge* __restrict__ in, unsigned long long* clk) {
    __shared__ geq qs[256];
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    ge r = in[i & 4095];
    const ge P = in[(i * 7 + 1) & 4095];
    {
        const fe ymx = fe_sub(P.Y, P.X), ypx = fe_add(P.Y, P.X);
#pragma unroll
        for (int k = 0; k < 4; k++) {
            qs[threadIdx.x].YmX.v[k] = ymx.v[k];
            qs[threadIdx.x].YpX.v[k] = ypx.v[k];
            qs[threadIdx.x].Z.v[k] = k ? 0 : 1;   // Z = 1: the ZONE forms, as for generators / normalized points
            qs[threadIdx.x].T.v[k] = P.T.v[k];
        }
    }
    uint64_t pat = 0x9E3779B97F4A7C15ull * (i + 1);
    const unsigned long long t0 = clock64(), w0 = wall_clock64();
    for (int s = 0; s < STEPS; s++) {
        if (KIND == 0) {
            const bool use_q = (pat & 3) == 0 || (pat & 12) == 0;   // per-lane mix of doublings and adds
            pat = (pat >> 1) | (pat << 63);
            r = ge_add_sel<true, true>(r, &qs[threadIdx.x], use_q);
        } else if (KIND == 1) {
            r = ge_dbl(r);
        } else {
            r = ge_add_qp<true>(r, &qs[threadIdx.x], true);
        }
    }
    const unsigned long long t1 = clock64(), w1 = wall_clock64();
    out[i] = r;
    if ((threadIdx.x & 63) == 0) {
        clk[2 * (i >> 6)] = t1 - t0;
        clk[2 * (i >> 6) + 1] = w1 - w0;
    }
}

template <int KIND>
void run(const char* name, ge* out, const ge* in, unsigned long long* dclk, int blocks, bool last) {
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    k_step<KIND><<<blocks, 256>>>(out, in, dclk);
    (void)hipDeviceSynchronize();
    (void)hipEventRecord(e0);
    k_step<KIND><<<blocks, 256>>>(out, in, dclk);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    const int waves = blocks * 4;
    std::vector<unsigned long long> h(2 * (size_t)waves);
    (void)hipMemcpy(h.data(), dclk, h.size() * 8, hipMemcpyDeviceToHost);
    double sc = 0, sr = 0;
    for (int k = 0; k < waves; k++) { sc += (double)h[2 * k]; sr += (double)h[2 * k + 1]; }
    int rate_khz = 0;
    (void)hipDeviceGetAttribute(&rate_khz, hipDeviceAttributeWallClockRate, 0);
    printf("  \"%s\": {\"ms\": %.4f, \"ghz\": %.4f, \"waves\": %d, \"steps_per_wave\": %d}%s\n", name, ms,
           sc / sr * rate_khz * 1e-6, waves, STEPS, last ? "" : ",");
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
}

int main() {
    hipDeviceProp_t p;
    (void)hipGetDeviceProperties(&p, 0);
    const int blocks = p.multiProcessorCount * 4;   // 4 blocks of 4 waves per CU: 4 waves per SIMD, one round
    std::vector<ge> h(4096);
    uint64_t x = 0x1234567;
    for (auto& g : h) {
        uint64_t* w = (uint64_t*)&g;
        for (int k = 0; k < 16; k++) {
            x = x * 6364136223846793005ull + 1442695040888963407ull;
            w[k] = x & (k % 4 == 3 ? 0x7FFFFFFFFFFFFFFFull : ~0ull);
        }
    }
    ge *din, *dout;
    unsigned long long* dclk;
    (void)hipMalloc(&din, 4096 * sizeof(ge));
    (void)hipMalloc(&dout, (size_t)blocks * 256 * sizeof(ge));
    (void)hipMalloc(&dclk, (size_t)blocks * 4 * 16);
    (void)hipMemcpy(din, h.data(), 4096 * sizeof(ge), hipMemcpyHostToDevice);
    printf("{\"device\": \"%s\", \"cus\": %d, \"waves_per_simd\": 4, \"kernels\": {\n", p.gcnArchName,
           p.multiProcessorCount);
    run<0>("step", dout, din, dclk, blocks, false);
    run<1>("dbl", dout, din, dclk, blocks, false);
    run<2>("add", dout, din, dclk, blocks, true);
    printf("}}\n");
    return 0;
}
