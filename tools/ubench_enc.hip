// ubench_enc.hip — issue cost of gfx950 VALU instructions by ENCODING (VOP1/VOP2 "e32" vs
// VOP3 "e64"), at 8 waves/SIMD with 8 independent chains per lane: which integer building
// blocks of the 256-bit limb arithmetic are full-rate.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define ITERS 16384
#define CH 8

#define OPS(X)                                                                                          \
    X(0, "v_add_u32_e32", "v_add_u32_e32 %0, %1, %0")                                                  \
    X(1, "v_add_u32_e64", "v_add_u32_e64 %0, %0, %1")                                                  \
    X(2, "v_and_b32_e32", "v_and_b32_e32 %0, %1, %0")                                                  \
    X(3, "v_or_b32_e32", "v_or_b32_e32 %0, %1, %0")                                                    \
    X(4, "v_xor_b32_e32", "v_xor_b32_e32 %0, %1, %0")                                                  \
    X(5, "v_lshlrev_b32_e32", "v_lshlrev_b32_e32 %0, 3, %0")                                          \
    X(6, "v_mov_b32_e32", "v_mov_b32_e32 %0, %1")                                                      \
    X(7, "v_sub_u32_e32", "v_sub_u32_e32 %0, %1, %0")                                                  \
    X(8, "v_alignbit_b32", "v_alignbit_b32 %0, %0, %1, 7")                                             \
    X(9, "v_lshl_or_b32", "v_lshl_or_b32 %0, %0, 3, %1")                                               \
    X(10, "v_or3_b32", "v_or3_b32 %0, %0, %1, %0")                                                     \
    X(11, "v_add_co_u32_e32(vcc)", "v_add_co_u32_e32 %0, vcc, %1, %0")                                 \
    X(12, "v_addc_co_u32_e32(vcc)", "v_addc_co_u32_e32 %0, vcc, 0, %0, vcc")                           \
    X(13, "v_addc_co_u32_e64(s)", "v_addc_co_u32_e64 %0, s[6:7], %0, 0, s[6:7]")                      \
    X(14, "v_cndmask_b32_e32(vcc)", "v_cndmask_b32_e32 %0, %1, %0, vcc")                               \
    X(15, "v_cndmask_b32_e64(s)", "v_cndmask_b32_e64 %0, %0, %1, s[6:7]")                              \
    X(16, "v_mad_u64_u32", "v_mad_u64_u32 %2, s[6:7], %0, %1, %2")                                    \
    X(17, "v_lshl_add_u64", "v_lshl_add_u64 %2, %2, 1, %2")                                           \
    X(18, "v_cmp_lt_u32_e32", "v_cmp_lt_u32_e32 vcc, %0, %1")                                          \
    X(19, "v_cmp_lt_u64_e64", "v_cmp_lt_u64_e64 s[6:7], %2, %2")                                      \
    X(20, "v_mul_lo_u32", "v_mul_lo_u32 %0, %0, %1")                                                   \
    X(21, "v_bfi_b32", "v_bfi_b32 %0, %0, %1, %0")                                                     \
    X(22, "v_perm_b32", "v_perm_b32 %0, %0, %1, %1")                                                   \
    X(23, "v_add3_u32", "v_add3_u32 %0, %0, %1, %0")                                                   \
    X(24, "v_subb_co_u32_e32(vcc)", "v_subb_co_u32_e32 %0, vcc, %1, %0, vcc")                          \
    X(25, "v_lshrrev_b64", "v_lshrrev_b64 %2, 3, %2")                                                  \
    X(26, "v_mov_b64", "v_mov_b64 %2, %2")                                                             \
    X(27, "v_pk_add_u16", "v_pk_add_u16 %0, %0, %1")                                                   \
    X(28, "v_mad_u32_u24", "v_mad_u32_u24 %0, %0, %1, %0")                                             \
    X(29, "v_mul_hi_u32", "v_mul_hi_u32 %0, %0, %1")

template <int OP>
__global__ __launch_bounds__(256) void k(uint32_t* out, uint32_t seed) {
    uint32_t a[CH], b[CH];
    uint64_t w[CH];
    for (int c = 0; c < CH; c++) { a[c] = seed * (threadIdx.x + c + 1); b[c] = a[c] ^ 0x9e3779b9u; w[c] = a[c]; }
    for (int it = 0; it < ITERS; it++) {
#pragma unroll
        for (int c = 0; c < CH; c++) {
#define X(id, name, text) if (OP == id) asm volatile(text : "+v"(a[c]) : "v"(b[c]), "v"(w[c]) : "vcc", "s6", "s7");
            OPS(X)
#undef X
        }
    }
    uint32_t r = 0;
    for (int c = 0; c < CH; c++) r += a[c] + b[c] + (uint32_t)w[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

template <int OP>
void run(const char* name, uint32_t* out, int blocks) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    k<OP><<<blocks, 256>>>(out, 3);
    hipDeviceSynchronize();
    hipEventRecord(e0);
    k<OP><<<blocks, 256>>>(out, 5);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    double waveinstr = (double)blocks * 4 * ITERS * CH;
    double simd_cyc = (ms * 1e-3) * 2.4e9 * 1024;
    printf("%-26s %7.3f ms  %5.2f cycles/wave-instr/SIMD (at 2.4 GHz)\n", name, ms, simd_cyc / waveinstr);
}

int main() {
    int blocks = 256 * 8;
    uint32_t* out;
    hipMalloc(&out, blocks * 256 * 4);
#define X(id, name, text) run<id>(name, out, blocks);
    OPS(X)
    OPS(X)
#undef X
    hipFree(out);
    return 0;
}
