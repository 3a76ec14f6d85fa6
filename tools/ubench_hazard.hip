// ubench_hazard.hip — what a dependent instruction and a hazard wait state cost ONE wave alone on a
// SIMD (the latency-bound regime of the row / quad forms: a one-proof call, a drain tick).
// Each kernel is one wave (64 threads, one block) running an unrolled sequence; cycles per
// sequence element come from clock64 (shader clock) inside the kernel.
//   add      dependent v_add_u32                         (the VALU dependent-issue latency)
//   add4     four independent v_add_u32 chains, interleaved (single-wave issue rate)
//   nop0     dependent v_add_u32 + s_nop 0               (the price of one wait state)
//   nop1     dependent v_add_u32 + s_nop 1               (two wait states)
//   carry    v_addc_co_u32 VCC chain + s_nop 0            (gfx950: a carry read >= 1 wait state
//                                                         after its VALU write)
//   carry2   two carry chains (VCC, an SGPR pair) interleaved, no nop
//   mad      dependent v_mad_u64_u32 (64-bit accumulate)
//   dpp      v_mov_b32_dpp chain + s_nop 1 (a DPP read >= 2 wait states after the VALU write)
//   lshl     dependent v_lshl_add_u64
// Prints one JSON object: cycles per element for each.
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

#define R4(x) x x x x
#define R32(x) R4(R4(x)) R4(R4(x))
#define ITERS 256

template <int KIND>
__global__ void k(uint32_t* out, unsigned long long* clk, uint32_t seed) {
    uint32_t a = seed + threadIdx.x, b = seed * 3 + 1, c = a ^ 5, d = b + 7, e = a + 11, f = b ^ 13;
    uint64_t m = a;
    __syncthreads();
    const unsigned long long t0 = clock64();
    for (int it = 0; it < ITERS; it++) {
        if (KIND == 0) asm volatile(R32("v_add_u32 %0, %0, %1\n\t") : "+v"(a) : "v"(b));
        if (KIND == 1)
            asm volatile(R32("v_add_u32 %0, %0, %4\n\tv_add_u32 %1, %1, %4\n\tv_add_u32 %2, %2, %4\n\tv_add_u32 %3, %3, %4\n\t")
                         : "+v"(a), "+v"(c), "+v"(d), "+v"(e) : "v"(b));
        if (KIND == 2) asm volatile(R32("v_add_u32 %0, %0, %1\n\ts_nop 0\n\t") : "+v"(a) : "v"(b));
        if (KIND == 3) asm volatile(R32("v_add_u32 %0, %0, %1\n\ts_nop 1\n\t") : "+v"(a) : "v"(b));
        if (KIND == 4)
            asm volatile("v_add_co_u32 %0, vcc, %0, %1\n\ts_nop 0\n\t" R32("v_addc_co_u32 %0, vcc, %0, %1, vcc\n\ts_nop 0\n\t")
                         : "+v"(a) : "v"(b) : "vcc");
        if (KIND == 5)
            asm volatile("v_add_co_u32 %0, vcc, %0, %2\n\tv_add_co_u32 %1, s[4:5], %1, %2\n\t"
                         R32("v_addc_co_u32 %0, vcc, %0, %2, vcc\n\tv_addc_co_u32 %1, s[4:5], %1, %2, s[4:5]\n\t")
                         : "+v"(a), "+v"(c) : "v"(b) : "vcc", "s4", "s5");
        if (KIND == 6) asm volatile(R32("v_mad_u64_u32 %0, s[4:5], %1, %2, %0\n\t") : "+v"(m) : "v"(b), "v"(f) : "s4", "s5");
        if (KIND == 7)
            asm volatile("s_nop 1\n\t" R32("v_mov_b32_dpp %0, %0 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\ts_nop 1\n\t")
                         : "+v"(a));
        if (KIND == 8) asm volatile(R32("v_lshl_add_u64 %0, %0, 1, %0\n\t") : "+v"(m));
    }
    const unsigned long long t1 = clock64();
    out[threadIdx.x] = a + c + d + e + (uint32_t)m + (uint32_t)(m >> 32);
    if (threadIdx.x == 0) *clk = t1 - t0;
}

template <int KIND>
double run(uint32_t* out, unsigned long long* dclk) {
    k<KIND><<<1, 64>>>(out, dclk, 3);
    (void)hipDeviceSynchronize();
    k<KIND><<<1, 64>>>(out, dclk, 5);
    (void)hipDeviceSynchronize();
    unsigned long long c = 0;
    (void)hipMemcpy(&c, dclk, 8, hipMemcpyDeviceToHost);
    return (double)c / (ITERS * 32.0);
}

int main() {
    uint32_t* out;
    unsigned long long* dclk;
    (void)hipMalloc(&out, 64 * 4);
    (void)hipMalloc(&dclk, 8);
    printf("{\"cycles_per_element\": {\"add\": %.2f, \"add4\": %.2f, \"nop0\": %.2f, \"nop1\": %.2f, \"carry\": %.2f, "
           "\"carry2\": %.2f, \"mad\": %.2f, \"dpp\": %.2f, \"lshl\": %.2f}}\n",
           run<0>(out, dclk), run<1>(out, dclk), run<2>(out, dclk), run<3>(out, dclk), run<4>(out, dclk),
           run<5>(out, dclk), run<6>(out, dclk), run<7>(out, dclk), run<8>(out, dclk));
    return 0;
}
