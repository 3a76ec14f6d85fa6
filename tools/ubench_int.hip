// ubench_int.hip — measures per-CU throughput of the integer VALU instructions a
// 256-bit limb multiply can be built from on gfx950 (decides the fe_mul design).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define ITERS 32768
#define CH 8   // independent chains per lane

template <int OP>
__global__ __launch_bounds__(256) void k(uint32_t* out, uint32_t seed) {
    uint32_t a[CH], b[CH];
    uint64_t acc[CH];
    double d[CH];
    for (int c = 0; c < CH; c++) { a[c] = seed * (threadIdx.x + c + 1); b[c] = a[c] ^ 0x9e3779b9u; acc[c] = a[c]; d[c] = (double)a[c]; }
    for (int it = 0; it < ITERS; it++) {
#pragma unroll
        for (int c = 0; c < CH; c++) {
            if (OP == 0) {        // v_mad_u64_u32 (no carry use)
                asm volatile("v_mad_u64_u32 %0, s[0:1], %1, %2, %0" : "+v"(acc[c]) : "v"(a[c]), "v"(b[c]) : "s0", "s1");
            } else if (OP == 1) { // v_mul_lo_u32
                asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(a[c]) : "v"(b[c]));
            } else if (OP == 2) { // v_mul_hi_u32
                asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(a[c]) : "v"(b[c]));
            } else if (OP == 3) { // v_mul_u32_u24
                asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(a[c]) : "v"(b[c]));
            } else if (OP == 4) { // v_add_co_u32 + v_addc_co_u32 (64-bit add)
                asm volatile("v_add_co_u32 %0, vcc, %0, %2\n\tv_addc_co_u32 %1, vcc, %1, %3, vcc" : "+v"(a[c]), "+v"(b[c]) : "v"(seed), "v"(seed) : "vcc");
            } else if (OP == 5) { // v_fma_f64
                asm volatile("v_fma_f64 %0, %0, %0, %0" : "+v"(d[c]));
            } else if (OP == 6) { // v_add_u32
                asm volatile("v_add_u32 %0, %0, %1" : "+v"(a[c]) : "v"(b[c]));
            } else if (OP == 7) { // v_mul_hi_u32_u24
                asm volatile("v_mul_hi_u32_u24 %0, %0, %1" : "+v"(a[c]) : "v"(b[c]));
            } else if (OP == 8) { // v_mad_u32_u24
                asm volatile("v_mad_u32_u24 %0, %0, %1, %0" : "+v"(a[c]) : "v"(b[c]));
            } else if (OP == 9) { // v_cndmask_b32
                asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(a[c]) : "v"(b[c]) : "vcc");
            } else if (OP == 10) { // v_lshl_add_u64 (gfx940+)
                asm volatile("v_lshl_add_u64 %0, %0, 0, %0" : "+v"(acc[c]));
            } else if (OP == 12) { // v_add3_u32
                asm volatile("v_add3_u32 %0, %0, %1, %0" : "+v"(a[c]) : "v"(b[c]));
            } else if (OP == 13) { // mad with carry-out consumed by addc
                asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0\n\tv_addc_co_u32 %1, vcc, %1, 0, vcc" : "+v"(acc[c]), "+v"(a[c]) : "v"(b[c]) : "vcc");
            } else if (OP == 14) { // v_alignbit_b32
                asm volatile("v_alignbit_b32 %0, %0, %1, 7" : "+v"(a[c]) : "v"(b[c]));
            } else if (OP == 15) { // v_cndmask with s-mask
                asm volatile("v_cndmask_b32 %0, %0, %1, s[4:5]" : "+v"(a[c]) : "v"(b[c]) : "s4","s5");
            } else if (OP == 11) { // v_mul_f64
                asm volatile("v_mul_f64 %0, %0, %0" : "+v"(d[c]));
            }
        }
    }
    uint32_t r = 0;
    for (int c = 0; c < CH; c++) r += a[c] + b[c] + (uint32_t)acc[c] + (uint32_t)(acc[c] >> 32) + (uint32_t)d[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

template <int OP>
void run(const char* name, int ops_per_iter, uint32_t* out, int blocks) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    k<OP><<<blocks, 256>>>(out, 3);
    hipDeviceSynchronize();
    hipEventRecord(e0);
    k<OP><<<blocks, 256>>>(out, 5);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    double waveinstr = (double)blocks * 4 * ITERS * CH * ops_per_iter;  // 4 waves per block
    double per_cu_cyc = (ms * 1e-3) * 2.4e9 * 256;   // CU-cycles at 2.4 GHz nominal
    printf("%-22s %8.3f ms  %7.2f wave-instr/CU/cycle  (%.2f cycles per wave-instr per SIMD)\n", name, ms,
           waveinstr / per_cu_cyc, 4.0 / (waveinstr / per_cu_cyc));
}

int main() {
    int blocks = 256 * 8;
    uint32_t* out; hipMalloc(&out, blocks * 256 * 4);
    run<6>("v_add_u32", 1, out, blocks);
    run<9>("v_cndmask_b32", 1, out, blocks);
    run<4>("v_add_co+v_addc (2)", 2, out, blocks);
    run<3>("v_mul_u32_u24", 1, out, blocks);
    run<7>("v_mul_hi_u32_u24", 1, out, blocks);
    run<8>("v_mad_u32_u24", 1, out, blocks);
    run<1>("v_mul_lo_u32", 1, out, blocks);
    run<2>("v_mul_hi_u32", 1, out, blocks);
    run<0>("v_mad_u64_u32", 1, out, blocks);
    run<10>("v_lshl_add_u64", 1, out, blocks);
    run<5>("v_fma_f64", 1, out, blocks);
    run<11>("v_mul_f64", 1, out, blocks);
    run<12>("v_add3_u32", 1, out, blocks);
    run<13>("mad_u64+addc (2)", 2, out, blocks);
    run<14>("v_alignbit_b32", 1, out, blocks);
    run<15>("v_cndmask(s)", 1, out, blocks);
    run<6>("v_add_u32 (again)", 1, out, blocks);
    hipFree(out);
    return 0;
}
