// ubench_issue.hip — VALU issue cost per wave64 instruction on gfx950, in SHADER CLOCK cycles
// (with LAT defined, ubench_lat: ONE wave per SIMD and one dependent chain, i.e. the latency)
// (the clock the VALU runs at, whatever the DVFS state), for the opcodes of the verify's hot loop.
//
// ubench_enc.hip priced instructions from wall time at a nominal 2.4 GHz; the k_terms PMC run
// then showed fewer cycles per instruction than that model (3.66 cycles per VALU
// instruction per SIMD at the PMC clock), so the nominal-clock costs overstate every cycle.
// Here each wave also reads the shader clock counter (clock64: s_memtime) and the constant
// 100 MHz counter (wall_clock64: s_memrealtime) around its loop: their ratio is the shader clock
// during the run, and wall time x that clock x 1024 SIMDs / wave-instructions is the issue cost.
// 8 waves per SIMD (2048 blocks of 256 on 256 CUs), 8 independent chains per lane (each with its own
// carry SGPR pair), so the cost is throughput, not latency.  Prints one JSON object: per opcode {cycles, ghz}.
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <vector>

#define ITERS 8192
#ifdef LAT
#define CH 1      // one chain ...
#define REP 16    // ... of 16 dependent copies per loop trip (the loop's own cost amortised)
#define WPS 1
#else
#define CH 8
#define REP 8
#define WPS 8
#endif

#define OPS(X)                                                                                       \
    X(0, "v_addc_co_u32", "v_addc_co_u32_e64 %0, %3, %0, %1, %3")                          \
    X(1, "v_mad_u64_u32", "v_mad_u64_u32 %2, %3, %0, %1, %2")                                    \
    X(2, "v_mov_b32", "v_mov_b32_e32 %0, %1")                                                         \
    X(3, "v_lshl_add_u64", "v_lshl_add_u64 %2, %2, 1, %2")                                            \
    X(4, "v_cndmask_b32", "v_cndmask_b32_e64 %0, %0, %1, %3")                                     \
    X(5, "v_cmp_eq_u32", "v_cmp_eq_u32_e64 %3, %0, %1")                                           \
    X(6, "v_add_co_u32", "v_add_co_u32_e64 %0, %3, %0, %1")                                       \
    X(7, "v_subb_co_u32", "v_subb_co_u32_e64 %0, %3, %0, %1, %3")                            \
    X(8, "v_add_u32", "v_add_u32_e32 %0, %1, %0")                                                     \
    X(9, "v_max3_u32", "v_max3_u32 %0, %0, %1, %0")                                                   \
    X(10, "v_max_u32", "v_max_u32_e32 %0, %1, %0")                                                    \
    X(11, "v_cmp_gt_i32", "v_cmp_gt_i32_e64 %3, %0, %1")                                          \
    X(12, "v_alignbit_b32", "v_alignbit_b32 %0, %0, %1, 7")                                           \
    X(13, "v_mov_b64", "v_mov_b64 %2, %2")                                                            \
    X(14, "v_sub_co_u32", "v_sub_co_u32_e64 %0, %3, %0, %1")                                      \
    X(15, "v_lshlrev_b32", "v_lshlrev_b32_e32 %0, 3, %0")                                             \
    X(16, "v_not_b32", "v_not_b32_e32 %0, %0")                                                        \
    X(17, "v_addc_co_u32_e32", "v_addc_co_u32_e32 %0, vcc, %1, %0, vcc")                              \
    X(18, "v_cndmask_b32_e32", "v_cndmask_b32_e32 %0, %1, %0, vcc")                                   \
    X(19, "v_fma_f64", "v_fma_f64 %2, %2, %2, %2")                                                    \
    X(20, "v_mul_lo_u32", "v_mul_lo_u32 %0, %0, %1")                                                  \
    X(21, "v_mul_hi_u32", "v_mul_hi_u32 %0, %0, %1")                                                  \
    X(22, "s_nop_0", "s_nop 0")                                                                        \
    X(23, "v_mov_b32_dpp", "v_mov_b32_dpp %0, %0 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf")         \
    X(24, "pair:mad+mov", "v_mad_u64_u32 %2, %3, %0, %1, %2\n\tv_mov_b32_e32 %0, %1")                    \
    X(25, "pair:mad+add_u32", "v_mad_u64_u32 %2, %3, %0, %1, %2\n\tv_add_u32_e32 %0, %1, %0")           \
    X(26, "pair:addc+mov", "v_addc_co_u32_e64 %0, %3, %0, %1, %3\n\tv_mov_b32_e32 %1, %0")               \
    X(27, "pair:mad+addc", "v_mad_u64_u32 %2, %3, %0, %1, %2\n\tv_addc_co_u32_e64 %0, %3, %0, %1, %3")   \
    X(28, "pair:mov+mov", "v_mov_b32_e32 %0, %1\n\tv_mov_b32_e32 %1, %0")                             \
    /* the guide's 2-cycle wave64 issue is an f32 figure (MI355X_MICROARCH.md, 'vector-instruction   */ \
    /* ISSUE cost': v_add_f32 / v_fma_f32); the same harness on them reconciles it with the integer */ \
    /* rows above (v_add_u32 ~3.4, VOP3 carry / 64-bit ops ~4.5)                                    */ \
    X(29, "v_add_f32", "v_add_f32_e32 %0, %1, %0")                                                     \
    X(30, "v_fma_f32", "v_fma_f32 %0, %0, %1, %0")                                                     \
    X(31, "v_mul_f32", "v_mul_f32_e32 %0, %1, %0")                                                     \
    X(32, "v_xor_b32", "v_xor_b32_e32 %0, %1, %0")                                                     \
    X(33, "v_add_co_u32_e32", "v_add_co_u32_e32 %0, vcc, %1, %0")

constexpr int NOPS = 34;

template <int OP>
__global__ __launch_bounds__(256) void k(uint32_t* out, unsigned long long* clk, uint32_t seed) {
    uint32_t a[CH], b[CH];
    uint64_t w[CH], sm[CH];
    for (int c = 0; c < CH; c++) {
        sm[c] = 0;
        a[c] = seed * (threadIdx.x + c + 1);
        b[c] = a[c] ^ 0x9e3779b9u;
        w[c] = a[c];
    }
    const unsigned long long t0 = clock64(), r0 = wall_clock64();
    for (int it = 0; it < ITERS; it++) {
#pragma unroll
        for (int r = 0; r < REP; r++) {
            const int c = r % CH;
#define X(id, name, text) \
    if (OP == id) asm volatile(text : "+v"(a[c]), "+v"(b[c]), "+v"(w[c]), "+s"(sm[c]) : : "vcc");
            OPS(X)
#undef X
        }
    }
    const unsigned long long t1 = clock64(), r1 = wall_clock64();
    uint32_t r = 0;
    for (int c = 0; c < CH; c++) r += a[c] + b[c] + (uint32_t)w[c] + (uint32_t)sm[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = r;
    if ((threadIdx.x & 63) == 0) {
        const size_t wv = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
        clk[2 * wv] = t1 - t0;
        clk[2 * wv + 1] = r1 - r0;
    }
}

template <int OP>
void run(const char* name, uint32_t* out, unsigned long long* dclk, int blocks, bool last) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    k<OP><<<blocks, 256>>>(out, dclk, 3);
    hipDeviceSynchronize();
    hipEventRecord(e0);
    k<OP><<<blocks, 256>>>(out, dclk, 5);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    const int waves = blocks * 4;
    std::vector<unsigned long long> h(2 * (size_t)waves);
    hipMemcpy(h.data(), dclk, h.size() * 8, hipMemcpyDeviceToHost);
    double sc = 0, sr = 0;
    for (int i = 0; i < waves; i++) { sc += (double)h[2 * i]; sr += (double)h[2 * i + 1]; }
    int rate_khz = 0;
    hipDeviceGetAttribute(&rate_khz, hipDeviceAttributeWallClockRate, 0);
    const double ghz = sc / sr * rate_khz * 1e-6;                 // shader clock during the loop
    const double winstr = (double)waves * ITERS * REP;
    const double cyc = (ms * 1e-3) * ghz * 1e9 * 1024 / winstr;   // issue cycles per wave-instr per SIMD
    printf("  \"%s\": {\"cycles\": %.3f, \"ghz\": %.4f, \"ms\": %.3f}%s\n", name, cyc, ghz, ms, last ? "" : ",");
    hipEventDestroy(e0);
    hipEventDestroy(e1);
}

template <int OP>
void run_all(uint32_t* out, unsigned long long* dclk, int blocks) {
    constexpr const char* names[] = {
#define X(id, name, text) name,
        OPS(X)
#undef X
    };
    run<OP>(names[OP], out, dclk, blocks, OP == NOPS - 1);
    if constexpr (OP + 1 < NOPS) run_all<OP + 1>(out, dclk, blocks);
}

int main() {
    hipDeviceProp_t p;
    hipGetDeviceProperties(&p, 0);
    const int blocks = p.multiProcessorCount * WPS;   // WPS blocks of 4 waves per CU = WPS waves per SIMD
    uint32_t* out;
    unsigned long long* dclk;
    hipMalloc(&out, (size_t)blocks * 256 * 4);
    hipMalloc(&dclk, (size_t)blocks * 4 * 16);
    printf("{\"device\": \"%s\", \"cus\": %d, \"waves_per_simd\": %d, \"chains\": %d, \"ops\": {\n", p.gcnArchName,
           p.multiProcessorCount, WPS, CH);
    run_all<0>(out, dclk, blocks);
    printf("}}\n");
    hipFree(out);
    hipFree(dclk);
    return 0;
}
