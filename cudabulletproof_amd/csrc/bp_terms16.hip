// bp_terms16.hip — the k_terms instantiation for QL = 16 (bp_verify_dev.h), a translation unit of its
// own so the large tick kernels compile in parallel.
#include <algorithm>

#include "bp_verify_dev.h"

namespace bp {

// The engine's table upload (bp_capi.hip Engine::upload): the kernel reads the pinned host staging
// buffer directly, so the first call's path issues no copy-engine transfer (a first hipMemcpyAsync of
// the 33-KB identity-doubling table cost ~7 ms; profiles/dropin_first_call_r05g.txt).  It lives in
// the row-form tick's code object, which a one-proof call loads anyway.
__global__ void k_upload(uint4* __restrict__ dst, const uint4* __restrict__ src, size_t n16) {
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += (size_t)gridDim.x * blockDim.x)
        dst[i] = src[i];
}
void launch_upload(void* dst, const void* src, size_t bytes, hipStream_t s) {
    const size_t n16 = bytes / 16;
    const unsigned blocks = (unsigned)std::min<size_t>((n16 + 255) / 256, 1024);
    if (n16) k_upload<<<blocks, 256, 0, s>>>((uint4*)dst, (const uint4*)src, n16);
}

void launch_terms16(const RegionList& rl, const SlotDev* slots, const ge* G, const ge* H, const ge* g,
                    const ge* h, const ge* dtab, const fe* two_i, hipStream_t s, unsigned lds_pad) {
    launch_terms_ql<16>(rl, slots, G, H, g, h, dtab, two_i, s, lds_pad);
}

}  // namespace bp
