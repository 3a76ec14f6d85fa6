// ubench_lat.hip — dependent-chain latency (1 wave per SIMD) and 2-wave/4-wave issue of
// v_mad_u64_u32 chains, to size ILP/occupancy needs of the limb multiply.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#define ITERS 65536
template <int CH>
__global__ void k(uint64_t* out, uint32_t seed) {
    uint64_t acc[CH];
    uint32_t a = seed * threadIdx.x + 1, b = a ^ 0x9e3779b9u;
    for (int c = 0; c < CH; c++) acc[c] = a + c;
    for (int it = 0; it < ITERS; it++) {
#pragma unroll
        for (int c = 0; c < CH; c++)
            asm volatile("v_mad_u64_u32 %0, s[0:1], %1, %2, %0" : "+v"(acc[c]) : "v"(a), "v"(b) : "s0", "s1");
    }
    uint64_t r = 0;
    for (int c = 0; c < CH; c++) r += acc[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}
template <int CH>
void run(int wps, uint64_t* out) {
    // one block of 64*4*wps threads per CU -> wps waves per SIMD
    int blocks = 256, threads = 256 * wps;
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
    k<CH><<<blocks, threads>>>(out, 3);
    (void)hipDeviceSynchronize();
    (void)hipEventRecord(e0);
    k<CH><<<blocks, threads>>>(out, 5);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms; (void)hipEventElapsedTime(&ms, e0, e1);
    double per_simd_instr = (double)ITERS * CH * wps;          // wave-instructions per SIMD
    double cyc = ms * 1e-3 * 2.4e9;
    printf("chains/lane=%d waves/SIMD=%d : %.2f cycles per wave-instr per SIMD (%.2f per chain step)\n", CH, wps,
           cyc / per_simd_instr, cyc / ITERS);
}
int main() {
    uint64_t* out; (void)hipMalloc(&out, 256 * 1024 * 8);
    run<1>(1, out); run<2>(1, out); run<4>(1, out); run<8>(1, out);
    run<1>(2, out); run<2>(2, out); run<1>(4, out); run<4>(4, out);
    return 0;
}
