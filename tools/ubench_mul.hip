// ubench_mul.hip — the exact 256x256 product in two forms, priced on gfx950:
//   col  product scanning (mul512_asm.h: v_mad_u64_u32 with SGPR carry-out + v_addc carry count)
//   row  operand scanning in C ((u64) a_i b_j + w_{i+j} + carry: v_mad_u64_u32 + the carry's add; the
//        carry cannot ride in the mad's 64-bit addend: w + carry << 32 has the wrong weight, and
//        w_{i+j+1} << 32 + carry overflows 64 bits)
// each followed by the same fold (fe_fold512), i.e. a whole fe_mul.  Throughput: 4 waves per SIMD
// (k_terms' occupancy), two independent chains per lane.  Latency: 1 wave per SIMD, one chain.
// Both forms' results are checked equal.  Prints one JSON object (cycles per fe_mul per SIMD).
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <vector>

#include "../cudabulletproof_amd/csrc/fe25519_dev.h"

using namespace bp;

#define ITERS 2048

__device__ __forceinline__ void mul512_row(uint64_t t[8], const fe& f, const fe& g) {
    uint32_t a[8], b[8], w[16];
#pragma unroll
    for (int i = 0; i < 4; i++) {
        a[2 * i] = (uint32_t)f.v[i];
        a[2 * i + 1] = (uint32_t)(f.v[i] >> 32);
        b[2 * i] = (uint32_t)g.v[i];
        b[2 * i + 1] = (uint32_t)(g.v[i] >> 32);
    }
    {
        uint32_t carry = 0;
#pragma unroll
        for (int j = 0; j < 8; j++) {
            const uint64_t p = (uint64_t)a[0] * b[j] + carry;
            w[j] = (uint32_t)p;
            carry = (uint32_t)(p >> 32);
        }
        w[8] = carry;
    }
#pragma unroll
    for (int i = 1; i < 8; i++) {
        uint32_t carry = 0;
#pragma unroll
        for (int j = 0; j < 8; j++) {
            const uint64_t p = (uint64_t)a[i] * b[j] + w[i + j] + carry;
            w[i + j] = (uint32_t)p;
            carry = (uint32_t)(p >> 32);
        }
        w[i + 8] = carry;
    }
#pragma unroll
    for (int i = 0; i < 8; i++) t[i] = (uint64_t)w[2 * i] | ((uint64_t)w[2 * i + 1] << 32);
}

template <int FORM>
__device__ __forceinline__ fe mulf(const fe& x, const fe& y) {
    uint64_t t[8];
    if (FORM == 0) mul512(t, x, y);
    else mul512_row(t, x, y);
    return fe_fold512(t);
}

template <int FORM, int CHAINS>
__global__ __launch_bounds__(256) void k(fe* out, const fe* in, unsigned long long* clk) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    fe x = in[i & 1023], y = in[(i * 7 + 3) & 1023], u = in[(i * 5 + 1) & 1023];
    const unsigned long long t0 = clock64(), w0 = wall_clock64();
    for (int s = 0; s < ITERS; s++) {
        x = mulf<FORM>(x, y);
        if (CHAINS == 2) u = mulf<FORM>(u, y);
    }
    const unsigned long long t1 = clock64(), w1 = wall_clock64();
    if (CHAINS == 2) {
#pragma unroll
        for (int k = 0; k < 4; k++) x.v[k] ^= u.v[k];
    }
    out[i] = x;
    if ((threadIdx.x & 63) == 0) {
        clk[2 * (i >> 6)] = t1 - t0;
        clk[2 * (i >> 6) + 1] = w1 - w0;
    }
}

template <int FORM, int CHAINS>
double run(fe* out, const fe* in, unsigned long long* dclk, int blocks, int tpb, std::vector<fe>& res) {
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    k<FORM, CHAINS><<<blocks, tpb>>>(out, in, dclk);
    (void)hipDeviceSynchronize();
    (void)hipEventRecord(e0);
    k<FORM, CHAINS><<<blocks, tpb>>>(out, in, dclk);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    const int waves = blocks * tpb / 64;
    std::vector<unsigned long long> h(2 * (size_t)waves);
    (void)hipMemcpy(h.data(), dclk, h.size() * 8, hipMemcpyDeviceToHost);
    res.resize((size_t)blocks * tpb);
    (void)hipMemcpy(res.data(), out, res.size() * sizeof(fe), hipMemcpyDeviceToHost);
    double sc = 0, sr = 0;
    for (int q = 0; q < waves; q++) { sc += (double)h[2 * q]; sr += (double)h[2 * q + 1]; }
    int rate_khz = 0;
    (void)hipDeviceGetAttribute(&rate_khz, hipDeviceAttributeWallClockRate, 0);
    const double ghz = sc / sr * rate_khz * 1e-6;
    // cycles per fe_mul per SIMD: wall cycles x 1024 SIMDs / (waves x muls per wave)
    const double muls = (double)waves * ITERS * CHAINS;
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    return (ms * 1e-3) * ghz * 1e9 * 1024 / muls;
}

int main() {
    hipDeviceProp_t p;
    (void)hipGetDeviceProperties(&p, 0);
    const int cus = p.multiProcessorCount;
    std::vector<fe> h(1024);
    uint64_t s = 0x1234567;
    for (auto& f : h)
        for (int q = 0; q < 4; q++) {
            s = s * 6364136223846793005ull + 1442695040888963407ull;
            f.v[q] = s & (q == 3 ? 0x7FFFFFFFFFFFFFFFull : ~0ull);
        }
    fe *din, *dout;
    unsigned long long* dclk;
    (void)hipMalloc(&din, 1024 * sizeof(fe));
    (void)hipMalloc(&dout, (size_t)cus * 4 * 256 * sizeof(fe));
    (void)hipMalloc(&dclk, (size_t)cus * 4 * 4 * 16);
    (void)hipMemcpy(din, h.data(), 1024 * sizeof(fe), hipMemcpyHostToDevice);
    std::vector<fe> r0, r1, l0, l1;
    // throughput: 4 blocks of 256 per CU = 4 waves per SIMD; latency: 4 blocks of 64 per CU = 1 wave per SIMD
    const double tc = run<0, 2>(dout, din, dclk, cus * 4, 256, r0), tr = run<1, 2>(dout, din, dclk, cus * 4, 256, r1);
    const double lc = run<0, 1>(dout, din, dclk, cus * 4, 64, l0), lr = run<1, 1>(dout, din, dclk, cus * 4, 64, l1);
    bool same = r0.size() == r1.size() && l0.size() == l1.size();
    for (size_t q = 0; same && q < r0.size(); q++) same = fe_eq(r0[q], r1[q]);
    for (size_t q = 0; same && q < l0.size(); q++) same = fe_eq(l0[q], l1[q]);
    printf("{\"device\": \"%s\", \"throughput_cycles_per_mul_per_simd\": {\"col\": %.1f, \"row\": %.1f}, "
           "\"latency_cycles_per_mul_1wave\": {\"col\": %.1f, \"row\": %.1f}, \"same_bits\": %s}\n",
           p.gcnArchName, tc, tr, lc * 1.0, lr * 1.0, same ? "true" : "false");
    return same ? 0 : 1;
}
