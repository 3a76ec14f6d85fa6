// asm_check.hip — device asm forms (field_asm.h) vs the C forms of fe25519_dev.h on the GPU,
// edge-heavy random inputs.  Build: hipcc --offload-arch=gfx950 -O3 tools/asm_check.hip
#define BP_FIELD_ASM 1
#include "../cudabulletproof_amd/csrc/ge25519_dev.h"
#include <cstdio>
#include <cstring>
#include <vector>
using namespace bp;

#define BP_C 1
namespace cref {   // the C forms compiled for the device too (asm disabled for this namespace)
}

__device__ fe c_add(const fe& f, const fe& g) {
    fe h; unsigned c = 0;
    for (int i = 0; i < 4; i++) {
        uint32_t l = __builtin_addc(lo32(f.v[i]), lo32(g.v[i]), c, &c);
        uint32_t u = __builtin_addc(hi32(f.v[i]), hi32(g.v[i]), c, &c);
        h.v[i] = cat64(l, u);
    }
    return fe_fix(h, c != 0);
}

__global__ void k(const fe* a, const fe* b, fe* o_asm, fe* o_c, int n) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    o_asm[i] = fe_add(a[i], b[i]);
    o_c[i] = c_add(a[i], b[i]);
}

static uint64_t st = 88172645463325252ull;
static uint64_t rnd() { st ^= st << 13; st ^= st >> 7; st ^= st << 17; return st; }
static uint64_t edge() {
    const uint64_t E[] = {0, 1, 19, 0xFFFFFFFFFFFFFFEDull, 0xFFFFFFFFFFFFFFFFull, 0x7FFFFFFFFFFFFFFFull, 0x8000000000000000ull};
    return (rnd() & 1) ? E[rnd() % 7] : rnd();
}

int main() {
    const int n = 1 << 16;
    std::vector<fe> a(n), b(n), oa(n), oc(n);
    for (int i = 0; i < n; i++) for (int j = 0; j < 4; j++) { a[i].v[j] = edge(); b[i].v[j] = edge(); }
    fe *da, *db, *dA, *dC;
    hipMalloc(&da, n * 32); hipMalloc(&db, n * 32); hipMalloc(&dA, n * 32); hipMalloc(&dC, n * 32);
    hipMemcpy(da, a.data(), n * 32, hipMemcpyHostToDevice);
    hipMemcpy(db, b.data(), n * 32, hipMemcpyHostToDevice);
    k<<<n / 256, 256>>>(da, db, dA, dC, n);
    hipError_t e = hipDeviceSynchronize();
    printf("sync: %s\n", hipGetErrorString(e));
    hipMemcpy(oa.data(), dA, n * 32, hipMemcpyDeviceToHost);
    hipMemcpy(oc.data(), dC, n * 32, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int i = 0; i < n; i++) bad += memcmp(&oa[i], &oc[i], 32) != 0;
    printf("add mismatches %d / %d\n", bad, n);
    return bad != 0;
}
