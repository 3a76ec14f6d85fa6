// hazard_probe.hip — is a VALU carry-out SGPR read back correctly by the next VALU carry-in at
// 0, 1 or 2 wait states?  (tools/gen_mul_asm.py / gen_field_asm.py space a carry-in read 1 wait
// state after its write, as the compiler pads its own e64 carry chains, and a mask / source read 2.)  Each sequence
// first zeroes the SGPR pair with SALU, then a VALU instruction writes carry = 1 into it in every
// lane, then after K wait states a v_addc_co_u32 reads it as its carry-in: 1 if it saw the VALU
// write, 0 if it read the stale SALU zero.  One wave alone (the tightest timing) and 4096 waves;
// prints the lanes x repetitions that read a stale carry, per form and K.  A probe, not a proof:
// the generators never go below the compiler's own spacing.
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

#define REPS 256
#define N0 ""
#define N1 "s_nop 0\n\t"
#define N2 "s_nop 1\n\t"

// FORM 0: v_add_co_u32 (VOP3b, SGPR carry-out) -> v_addc_co_u32 carry-in
// FORM 1: v_mad_u64_u32 (SGPR carry-out of the 64-bit accumulate) -> v_addc_co_u32 carry-in
// FORM 2: v_add_co_u32_e32 (VCC) -> v_addc_co_u32_e32 (VCC carry-in)
#define SEQ0(NOP)                                                                                          \
    asm volatile("s_mov_b64 s[20:21], 0\n\tv_add_co_u32 %0, s[20:21], %1, %2\n\t" NOP                       \
                 "v_addc_co_u32 %0, s[22:23], 0, 0, s[20:21]"                                             \
                 : "=&v"(got) : "v"(ones), "v"(one) : "s20", "s21", "s22", "s23")
#define SEQ1(NOP)                                                                                          \
    asm volatile("s_mov_b64 s[20:21], 0\n\tv_mad_u64_u32 %1, s[20:21], %2, %2, %1\n\t" NOP                  \
                 "v_addc_co_u32 %0, s[22:23], 0, 0, s[20:21]"                                             \
                 : "=&v"(got), "+v"(acc) : "v"(one) : "s20", "s21", "s22", "s23")
#define SEQ2(NOP)                                                                                          \
    asm volatile("s_mov_b64 vcc, 0\n\tv_add_co_u32_e32 %0, vcc, %1, %2\n\t" NOP                            \
                 "v_addc_co_u32_e32 %0, vcc, 0, %3, vcc"                                                  \
                 : "=&v"(got) : "v"(ones), "v"(one), "v"(zero) : "vcc")

template <int FORM, int K>
__global__ void k_probe(unsigned* stale, uint32_t ones_in) {
    unsigned bad = 0;
    const uint32_t ones = ones_in, one = 1u, zero = 0u;
    for (int r = 0; r < REPS; r++) {
        uint32_t got = 0;
        uint64_t acc = ~0ull;   // + 1 * 1 carries out of 64 bits
        if (FORM == 0) { if (K == 0) SEQ0(N0); else if (K == 1) SEQ0(N1); else SEQ0(N2); }
        if (FORM == 1) { if (K == 0) SEQ1(N0); else if (K == 1) SEQ1(N1); else SEQ1(N2); }
        if (FORM == 2) { if (K == 0) SEQ2(N0); else if (K == 1) SEQ2(N1); else SEQ2(N2); }
        bad += got != 1u;
        (void)acc;
    }
    if (bad) atomicAdd(stale, bad);
}

template <int FORM, int K>
void run(unsigned* d, const char* name) {
    unsigned h[2] = {0, 0};
    (void)hipMemset(d, 0, 8);
    k_probe<FORM, K><<<1, 64>>>(d, 0xFFFFFFFFu);
    k_probe<FORM, K><<<1024, 256>>>(d + 1, 0xFFFFFFFFu);
    (void)hipDeviceSynchronize();
    (void)hipMemcpy(h, d, 8, hipMemcpyDeviceToHost);
    printf("%s\"%s_k%d\": {\"one_wave\": %u, \"many_waves\": %u}", (FORM || K) ? ", " : "", name, K, h[0], h[1]);
}

int main() {
    unsigned* d;
    (void)hipMalloc(&d, 8);
    printf("{\"stale_reads\": {");
    run<0, 0>(d, "add_co_e64"); run<0, 1>(d, "add_co_e64"); run<0, 2>(d, "add_co_e64");
    run<1, 0>(d, "mad_u64"); run<1, 1>(d, "mad_u64"); run<1, 2>(d, "mad_u64");
    run<2, 0>(d, "add_co_vcc"); run<2, 1>(d, "add_co_vcc"); run<2, 2>(d, "add_co_vcc");
    printf("}, \"reads_per_run\": {\"one_wave\": %d, \"many_waves\": %d}}\n", 64 * REPS, 1024 * 256 * REPS);
    return 0;
}
