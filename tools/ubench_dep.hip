// ubench_dep.hip — dependent-issue cost of instruction pairs for ONE wave alone on its SIMD (the
// row / quad forms' regime): each element is "producer; consumer that reads the producer's result",
// chained so every element depends on the one before.  Prints cycles per element (clock64);
// subtract the 4-cycle issue of each instruction to see the stall a dependency adds.
//   add_add   v_add_u32 -> v_add_u32                       (baseline: 2 instructions)
//   dpp_add   v_mov_b32_dpp -> v_add_u32 reading it
//   add_dpp   v_add_u32 -> s_nop 1 -> v_mov_b32_dpp reading it (the 2 required wait states)
//   mad_hi    v_mad_u64_u32 -> v_add_u32 reading its high half
//   mad_mad   v_mad_u64_u32 -> v_mad_u64_u32 accumulating it
//   lsh_lsh   v_lshl_add_u64 -> v_lshl_add_u64
//   addc_v    v_addc_co_u32 (VOP3b) -> v_addc_co_u32 reading its VGPR result (carry from elsewhere)
//   cmp_cnd   v_cmp_eq_u32 (VCC) -> s_nop 1 -> v_cndmask_b32 reading VCC
//   gate      v_cmp_eq_u32 (SGPR) -> s_cmp_lg_u64 -> s_cbranch_scc1 (the field asm's rare-edge test),
//             right after the compare or 8 independent VALU later, each against the same VALU ungated
//   and carry chains: VOP2 through VCC, VOP3b through an SGPR pair; independent VOP3b / VOP2 adds
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

#define R8(x) x x x x x x x x
#define R32(x) R8(x) R8(x) R8(x) R8(x)
#define ITERS 256

template <int KIND>
__global__ void k(uint32_t* out, unsigned long long* clk, uint32_t seed) {
    uint32_t a = seed + threadIdx.x, b = seed * 3 + 1;
    uint64_t m = a;
    uint32_t h2 = 0;
    __syncthreads();
    const unsigned long long t0 = clock64();
    for (int it = 0; it < ITERS; it++) {
        if (KIND == 0) asm volatile(R32("v_add_u32 %0, %0, %1\n\tv_add_u32 %0, %0, %1\n\t") : "+v"(a) : "v"(b));
        if (KIND == 1)
            asm volatile(R32("v_mov_b32_dpp %0, %0 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\tv_add_u32 %0, %0, %1\n\ts_nop 1\n\t")
                         : "+v"(a) : "v"(b));
        if (KIND == 2)
            asm volatile(R32("v_add_u32 %0, %0, %1\n\ts_nop 1\n\tv_mov_b32_dpp %0, %0 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t")
                         : "+v"(a) : "v"(b));
        if (KIND == 3) {
            uint32_t h;
            asm volatile(R32("v_mad_u64_u32 %1, s[4:5], %0, %2, %1\n\tv_add_u32 %0, %0, %3\n\t")
                         : "+v"(a), "+v"(m) : "v"(b), "v"(b) : "s4", "s5");
            (void)h;
        }
        if (KIND == 4) asm volatile(R32("v_mad_u64_u32 %0, s[4:5], %1, %2, %0\n\tv_mad_u64_u32 %0, s[4:5], %1, %2, %0\n\t") : "+v"(m) : "v"(a), "v"(b) : "s4", "s5");
        if (KIND == 5) asm volatile(R32("v_lshl_add_u64 %0, %0, 1, %0\n\tv_lshl_add_u64 %0, %0, 1, %0\n\t") : "+v"(m));
        if (KIND == 6)
            asm volatile("s_mov_b64 s[4:5], 0\n\t" R32("v_addc_co_u32 %0, s[6:7], %0, %1, s[4:5]\n\tv_addc_co_u32 %0, s[6:7], %0, %1, s[4:5]\n\t")
                         : "+v"(a) : "v"(b) : "s4", "s5", "s6", "s7");
        if (KIND == 8)   // VOP2 carry chain through VCC (carry and VGPR dependent)
            asm volatile("v_add_co_u32_e32 %0, vcc, %0, %1\n\t" R32("v_addc_co_u32_e32 %0, vcc, %0, %1, vcc\n\tv_addc_co_u32_e32 %0, vcc, %0, %1, vcc\n\t")
                         : "+v"(a) : "v"(b) : "vcc");
        if (KIND == 9)   // VOP3b carry chain through an SGPR pair (carry and VGPR dependent, 1 wait state)
            asm volatile("v_add_co_u32 %0, s[6:7], %0, %1\n\ts_nop 0\n\t" R32("v_addc_co_u32 %0, s[6:7], %0, %1, s[6:7]\n\ts_nop 0\n\tv_addc_co_u32 %0, s[6:7], %0, %1, s[6:7]\n\ts_nop 0\n\t")
                         : "+v"(a) : "v"(b) : "s6", "s7");
        if (KIND == 10)  // independent VOP3b adds (no dependency): the issue cost alone
            asm volatile(R32("v_add_co_u32 %0, s[6:7], %1, %1\n\tv_add_co_u32 %2, s[8:9], %1, %1\n\t")
                         : "=&v"(a), "+v"(b), "=&v"(h2) : : "s6", "s7", "s8", "s9");
        if (KIND == 11)  // independent VOP2 adds with VCC carry-out
            asm volatile(R32("v_add_co_u32_e32 %0, vcc, %1, %1\n\tv_add_co_u32_e32 %2, vcc, %1, %1\n\t")
                         : "=&v"(a), "+v"(b), "=&v"(h2) : : "vcc");
        if (KIND == 7)
            asm volatile(R32("v_cmp_eq_u32 vcc, %0, %1\n\ts_nop 1\n\tv_cndmask_b32 %0, %0, %1, vcc\n\t") : "+v"(a) : "v"(b) : "vcc");
        if (KIND == 12)  // rare-edge gate as the generated asm has it: VALU compare -> SALU test -> branch
            asm volatile(R32("v_cmp_eq_u32 s[4:5], -1, %0\n\ts_cmp_lg_u64 s[4:5], 0\n\ts_cbranch_scc1 1f\n1:\n\tv_add_u32 %0, %0, %1\n\t")
                         : "+v"(a) : "v"(b) : "s4", "s5", "scc");
        if (KIND == 13)  // the same compare without the SALU test and branch
            asm volatile(R32("v_cmp_eq_u32 s[4:5], -1, %0\n\tv_add_u32 %0, %0, %1\n\t") : "+v"(a) : "v"(b) : "s4", "s5");
        if (KIND == 14)  // gate with 8 independent VALU between the compare and the SALU test
            asm volatile(R32("v_cmp_eq_u32 s[4:5], -1, %0\n\t" R8("v_add_u32 %2, %2, %1\n\t") "s_cmp_lg_u64 s[4:5], 0\n\ts_cbranch_scc1 1f\n1:\n\tv_add_u32 %0, %0, %1\n\t")
                         : "+v"(a), "+v"(b), "+v"(h2) : : "s4", "s5", "scc");
        if (KIND == 16)  // compare into VCC -> s_cbranch_vccnz directly (no SALU test)
            asm volatile(R32("v_cmp_eq_u32_e32 vcc, -1, %0\n\ts_cbranch_vccnz 1f\n1:\n\tv_add_u32 %0, %0, %1\n\t")
                         : "+v"(a) : "v"(b) : "vcc");
        if (KIND == 17)  // compare into VCC, 8 independent VALU, s_cbranch_vccnz
            asm volatile(R32("v_cmp_eq_u32_e32 vcc, -1, %0\n\t" R8("v_add_u32 %2, %2, %1\n\t") "s_cbranch_vccnz 1f\n1:\n\tv_add_u32 %0, %0, %1\n\t")
                         : "+v"(a), "+v"(b), "+v"(h2) : : "vcc");
        if (KIND == 18)  // SALU test + branch on an SGPR no VALU wrote (the branch's own cost)
            asm volatile("s_mov_b64 s[4:5], 0\n\t" R32("s_cmp_lg_u64 s[4:5], 0\n\ts_cbranch_scc1 1f\n1:\n\tv_add_u32 %0, %0, %1\n\t")
                         : "+v"(a) : "v"(b) : "s4", "s5", "scc");
        if (KIND == 19)  // VALU compare -> SALU op reading it, no branch
            asm volatile("s_mov_b64 s[6:7], 0\n\t" R32("v_cmp_eq_u32 s[4:5], -1, %0\n\ts_or_b64 s[6:7], s[6:7], s[4:5]\n\tv_add_u32 %0, %0, %1\n\t")
                         : "+v"(a) : "v"(b) : "s4", "s5", "s6", "s7", "scc");
        if (KIND == 20)  // gate with 16 independent VALU between the compare and the SALU test
            asm volatile(R32("v_cmp_eq_u32 s[4:5], -1, %0\n\t" R8("v_add_u32 %2, %2, %1\n\tv_add_u32 %2, %2, %1\n\t") "s_cmp_lg_u64 s[4:5], 0\n\ts_cbranch_scc1 1f\n1:\n\tv_add_u32 %0, %0, %1\n\t")
                         : "+v"(a), "+v"(b), "+v"(h2) : : "s4", "s5", "scc");
        if (KIND == 21)  // the same 18 VALU without the gate
            asm volatile(R32("v_cmp_eq_u32 s[4:5], -1, %0\n\t" R8("v_add_u32 %2, %2, %1\n\tv_add_u32 %2, %2, %1\n\t") "v_add_u32 %0, %0, %1\n\t")
                         : "+v"(a), "+v"(b), "+v"(h2) : : "s4", "s5");
        if (KIND == 22)  // only a not-taken s_cbranch_scc1 (SCC from a SALU op long before)
            asm volatile("s_cmp_eq_u32 0, 1\n\t" R32("s_cbranch_scc1 1f\n1:\n\tv_add_u32 %0, %0, %1\n\t") : "+v"(a) : "v"(b) : "scc");
        if (KIND == 23)  // only a taken s_branch to the next instruction
            asm volatile(R32("s_branch 1f\n1:\n\tv_add_u32 %0, %0, %1\n\t") : "+v"(a) : "v"(b));
        if (KIND == 15)  // the same 10 VALU without the gate
            asm volatile(R32("v_cmp_eq_u32 s[4:5], -1, %0\n\t" R8("v_add_u32 %2, %2, %1\n\t") "v_add_u32 %0, %0, %1\n\t")
                         : "+v"(a), "+v"(b), "+v"(h2) : : "s4", "s5");
    }
    const unsigned long long t1 = clock64();
    out[threadIdx.x] = a + (uint32_t)m + h2;
    if (threadIdx.x == 0) *clk = t1 - t0;
}

template <int KIND>
double run(uint32_t* out, unsigned long long* d) {
    k<KIND><<<1, 64>>>(out, d, 3);
    (void)hipDeviceSynchronize();
    k<KIND><<<1, 64>>>(out, d, 5);
    (void)hipDeviceSynchronize();
    unsigned long long c = 0;
    (void)hipMemcpy(&c, d, 8, hipMemcpyDeviceToHost);
    return (double)c / (ITERS * 32.0);
}

int main() {
    uint32_t* out;
    unsigned long long* d;
    (void)hipMalloc(&out, 256);
    (void)hipMalloc(&d, 8);
    printf("{\"cycles_per_element\": {\"add_add\": %.2f, \"dpp_add_nop1\": %.2f, \"add_nop1_dpp\": %.2f, \"mad_hi\": %.2f, "
           "\"mad_mad\": %.2f, \"lsh_lsh\": %.2f, \"addc_v\": %.2f, \"cmp_nop1_cnd\": %.2f, \"addc_vcc_e32_chain\": %.2f, "
           "\"addc_sgpr_e64_chain_nop0\": %.2f, \"add_co_e64_indep\": %.2f, \"add_co_e32_indep\": %.2f, "
           "\"gate_cmp_scmp_br_add\": %.2f, \"cmp_add\": %.2f, \"gate_8indep\": %.2f, \"cmp_8indep_add\": %.2f, "
           "\"vcc_br_add\": %.2f, \"vcc_8indep_br_add\": %.2f, \"salu_scmp_br_add\": %.2f, \"cmp_sor_add\": %.2f, "
           "\"gate_16indep\": %.2f, \"cmp_16indep_add\": %.2f, \"br_add\": %.2f, \"sbranch_add\": %.2f}}\n",
           run<0>(out, d), run<1>(out, d), run<2>(out, d), run<3>(out, d), run<4>(out, d), run<5>(out, d),
           run<6>(out, d), run<7>(out, d), run<8>(out, d), run<9>(out, d), run<10>(out, d), run<11>(out, d),
           run<12>(out, d), run<13>(out, d), run<14>(out, d), run<15>(out, d),
           run<16>(out, d), run<17>(out, d), run<18>(out, d), run<19>(out, d), run<20>(out, d), run<21>(out, d), run<22>(out, d), run<23>(out, d));
    return 0;
}
