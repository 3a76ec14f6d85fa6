// bp_terms1.hip — the k_terms instantiation for QL = 1 (bp_verify_dev.h), a translation unit of its own so
// the large tick kernels compile in parallel.
#include "bp_verify_dev.h"

namespace bp {

void launch_terms1(const RegionList& rl, const SlotDev* slots, const ge* G, const ge* H, const ge* g,
                    const ge* h, const ge* dtab, const fe* two_i, hipStream_t s, unsigned lds_pad) {
    launch_terms_ql<1>(rl, slots, G, H, g, h, dtab, two_i, s, lds_pad);
}

}  // namespace bp
