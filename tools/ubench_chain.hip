// ubench_chain.hip — single-wave latency of the field building blocks the latency-bound forms
// (16-lane rows, lane quads) chain: each kernel is ONE wave looping x = op(x, ...) ITERS times,
// so every iteration waits for the previous one.  Prints cycles per iteration (clock64); against
// the blocks' static issue slots (VALU + wait states, tools/isa_count.py's probes) it gives the
// cost of one issue slot of a wave alone on its SIMD (profiles/ubench/ubench_chain_r06.json).
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

#include "../cudabulletproof_amd/csrc/ge25519_dev.h"
#include "../cudabulletproof_amd/csrc/ge25519_quad.h"

using namespace bp;

#define ITERS 2048

template <int KIND>
__global__ void c_chain(fe* out, const fe* in, unsigned long long* clk) {
    fe x = in[threadIdx.x], y = in[threadIdx.x + 64];
    uint32_t w[10];
    for (int i = 0; i < 10; i++) w[i] = (uint32_t)(x.v[i & 3] >> (8 * (i & 1)));
    const unsigned long long t0 = clock64();
    for (int it = 0; it < ITERS; it++) {
        if (KIND == 0) x = fe_mul(x, y);                 // one-lane product (the quad forms' stage)
        if (KIND == 1) x = fe_mul_q4(x, y);              // quad-split product (the row form's stage)
        if (KIND == 2) x = fe_mul_q4_k(x);               // quad-split product by k
        if (KIND == 3) x = fe_add(x, y);
        if (KIND == 4) { fe s, d; fe_addsub(x, y, s, d); x = fe_sel(threadIdx.x & 1, s, d); }
        if (KIND == 5) x = fe_row_bcast<4>(x);           // 8 DPP moves
        if (KIND == 6) {                                 // the quad sum + fold alone
            x = fe_q4_sum_fold(w);
            w[0] = (uint32_t)x.v[0]; w[3] = (uint32_t)x.v[1]; w[6] = (uint32_t)x.v[2]; w[9] = (uint32_t)x.v[3];
        }
        if (KIND == 7) {                                 // the fold alone
            uint64_t t[8] = {x.v[0], x.v[1], x.v[2], x.v[3], y.v[0], y.v[1], x.v[0] ^ y.v[2], y.v[3]};
            x = fe_fold512(t);
        }
        if (KIND == 8) x = fe_sq(x);
        if (KIND == 9) x = row_of_next(ge_row_of_step(x, fe_sel(threadIdx.x & 16, y, x)));   // the row step
    }
    const unsigned long long t1 = clock64();
    out[threadIdx.x] = x;
    if (threadIdx.x == 0) clk[KIND] = t1 - t0;
}

int main() {
    fe *din, *dout;
    unsigned long long* dclk;
    (void)hipMalloc(&din, 128 * sizeof(fe));
    (void)hipMalloc(&dout, 64 * sizeof(fe));
    (void)hipMalloc(&dclk, 16 * 8);
    fe h[128];
    uint64_t s = 0x243F6A8885A308D3ull;
    for (auto& f : h)
        for (int k = 0; k < 4; k++) {
            s ^= s << 13; s ^= s >> 7; s ^= s << 17;
            f.v[k] = k == 3 ? s >> 1 : s;
        }
    (void)hipMemcpy(din, h, sizeof h, hipMemcpyHostToDevice);
#define RUN(K) c_chain<K><<<1, 64>>>(dout, din, dclk); c_chain<K><<<1, 64>>>(dout, din, dclk);
    RUN(0) RUN(1) RUN(2) RUN(3) RUN(4) RUN(5) RUN(6) RUN(7) RUN(8) RUN(9)
    (void)hipDeviceSynchronize();
    unsigned long long c[16];
    (void)hipMemcpy(c, dclk, sizeof c, hipMemcpyDeviceToHost);
    const char* names[] = {"fe_mul", "fe_mul_q4", "fe_mul_q4_k", "fe_add", "fe_addsub+sel", "row_bcast",
                           "q4_sum_fold", "fold512", "fe_sq", "row_step"};
    printf("{\"cycles_per_iter\": {");
    for (int k = 0; k < 10; k++) printf("%s\"%s\": %.1f", k ? ", " : "", names[k], (double)c[k] / ITERS);
    printf("}}\n");
    return 0;
}
