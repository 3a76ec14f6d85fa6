// host_lanes_check.hip — TEST INFRASTRUCTURE (tests/test_host_arith.py).
//
// Compiles the verify pipeline's stage-0 lane layout (cudabulletproof_amd/csrc/bp_kernels.h:
// stage0_lanes / stage0_item, __host__ __device__) as HOST code and checks the split stage 0
// (Pipeline "deferred MSM terms", hipbp_pipeline_defer_msm): over every shape, with and without a
// lane order (perm0, as the lane sort writes it: a permutation within each per-lane class), the
// items reached by the S0_CRIT lanes (RK_STAGE0 of a split batch) and by the S0_DEFER lanes
// (RK_MSMT) are exactly the items of the unsplit stage 0, each once; the split's first part holds
// only fold round 0 and the polynomial terms, the second only the MSM terms, t*h and c*Q.
// Prints "<cases> <failures>"; exit status 1 on any failure.
#include <algorithm>
#include <cstdio>
#include <numeric>
#include <random>
#include <vector>

#include "../cudabulletproof_amd/csrc/bp_kernels.h"

using namespace bp;

static std::vector<uint32_t> items_of(const SlotDev& sd, int sel) {
    const Stage0Lanes z = stage0_lanes((unsigned long long)sd.bv.B, sd.bv.n, sd.bv.L_len, sd.range_mode, sel);
    std::vector<uint32_t> out;
    for (uint32_t l = 0; l < (uint32_t)z.total; l++) {
        const uint32_t it = stage0_item(sd, l, sel);
        if (it != UINT32_MAX) out.push_back(it);
    }
    return out;
}

int main() {
    int cases = 0, fails = 0;
    std::mt19937 rng(7);
    for (int mode = 0; mode <= 2; mode++)
        for (int n : {1, 2, 4, 16, 32, 64, 128})
            for (int B : {1, 3, 64, 70})
                for (int permuted = 0; permuted <= 1; permuted++) {
                    SlotDev sd{};
                    sd.bv.B = B;
                    sd.bv.n = n;
                    sd.bv.L_len = __builtin_ctz((unsigned)n);
                    sd.range_mode = mode;
                    const Stage0Lanes za = stage0_lanes(B, n, sd.bv.L_len, mode);
                    std::vector<uint32_t> perm(za.pl);
                    if (permuted) {   // a permutation within each class range, as launch_lane_sort writes
                        unsigned long long base = 0;
                        for (int c = 0; c < 4; c++) {
                            std::iota(perm.begin() + base, perm.begin() + base + za.size[c], 0u);
                            std::shuffle(perm.begin() + base, perm.begin() + base + za.size[c], rng);
                            base += za.size[c];
                        }
                        sd.perm0 = perm.data();
                    }
                    const uint32_t nA = mode ? 2u * n * B : 0, nB = sd.bv.L_len > 0 ? 2u * n * B : 0;
                    const uint32_t want = nA + nB + 2u * B + (mode == 2 ? 7u * B : 0);
                    std::vector<uint32_t> all = items_of(sd, S0_ALL), crit = items_of(sd, S0_CRIT),
                                          def = items_of(sd, S0_DEFER);
                    bool ok = all.size() == want;
                    for (uint32_t it : crit) ok &= (it >= nA && it < nA + nB) || it >= nA + nB + 2u * B;
                    for (uint32_t it : def) ok &= it < nA || (it >= nA + nB && it < nA + nB + 2u * B);
                    std::vector<uint32_t> u(crit);
                    u.insert(u.end(), def.begin(), def.end());
                    std::sort(all.begin(), all.end());
                    std::sort(u.begin(), u.end());
                    ok &= u == all && std::adjacent_find(all.begin(), all.end()) == all.end();
                    cases++;
                    if (!ok) {
                        fails++;
                        std::printf("FAIL mode %d n %d B %d permuted %d: all %zu crit %zu defer %zu want %u\n", mode, n,
                                    B, permuted, all.size(), crit.size(), def.size(), want);
                    }
                }
    std::printf("%d %d\n", cases, fails);
    return fails ? 1 : 0;
}
