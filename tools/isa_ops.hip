// isa_ops.hip — instruction-count probes (tools/isa_count.py): one field / point operation
// per kernel, compiled for gfx950, so the VALU cost of each building block can be tracked.
#include "../cudabulletproof_amd/csrc/ge25519_dev.h"
using namespace bp;
extern "C" __global__ void p_fe_add(fe* o, const fe* a, const fe* b) { o[threadIdx.x] = fe_add(a[threadIdx.x], b[threadIdx.x]); }
extern "C" __global__ void p_fe_sub(fe* o, const fe* a, const fe* b) { o[threadIdx.x] = fe_sub(a[threadIdx.x], b[threadIdx.x]); }
extern "C" __global__ void p_fe_mul(fe* o, const fe* a, const fe* b) { o[threadIdx.x] = fe_mul(a[threadIdx.x], b[threadIdx.x]); }
extern "C" __global__ void p_fe_fold(fe* o, const uint64_t* t) {
    uint64_t x[8];
    for (int i = 0; i < 8; i++) x[i] = t[threadIdx.x * 8 + i];
    o[threadIdx.x] = fe_fold512(x);
}
extern "C" __global__ void p_ge_dbl(ge* o, const ge* p) { o[threadIdx.x] = ge_dbl(p[threadIdx.x]); }
extern "C" __global__ void p_ge_add_q(ge* o, const ge* p, const geq* q) { o[threadIdx.x] = ge_add_q(p[threadIdx.x], q[threadIdx.x]); }
extern "C" __global__ void p_ge_add_sel(ge* o, const ge* p, const geq* q, const int* u) {
    __shared__ geq qs[256];
    qs[threadIdx.x] = q[threadIdx.x];
    o[threadIdx.x] = ge_add_sel<true>(p[threadIdx.x], &qs[threadIdx.x], u[threadIdx.x] != 0);
}
extern "C" __global__ void p_fe_sq(fe* o, const fe* a) { o[threadIdx.x] = fe_sq(a[threadIdx.x]); }
extern "C" __global__ void p_ge_add_zone(ge* o, const ge* p, const geq* q) {
    __shared__ geq qs[256];
    qs[threadIdx.x] = q[threadIdx.x];
    o[threadIdx.x] = ge_add_qp<true>(p[threadIdx.x], &qs[threadIdx.x], true);
}
extern "C" __global__ void p_ge_add_sel_zone(ge* o, const ge* p, const geq* q, const int* u) {
    __shared__ geq qs[256];
    qs[threadIdx.x] = q[threadIdx.x];
    o[threadIdx.x] = ge_add_sel<true, true>(p[threadIdx.x], &qs[threadIdx.x], u[threadIdx.x] != 0);
}
extern "C" __global__ void p_fe_canon(fe* o, const fe* a) { o[threadIdx.x] = fe_canon(a[threadIdx.x]); }
// one step of the drain-tick forms (sm_quad / sm_pair loop bodies): the latency-bound chains
#include "../cudabulletproof_amd/csrc/ge25519_quad.h"
extern "C" __global__ void p_quad_step(ge* o, const ge* p, const fe* qs, const int* u) {
    const int qd = threadIdx.x & 3;
    const ge r = p[threadIdx.x];
    const fe x1 = fe_sel4(qd, fe_sub(r.Y, r.X), fe_add(r.Y, r.X), r.T, r.Z);
    o[threadIdx.x] = ge_quad_finish(fe_mul(x1, fe_sel(u[threadIdx.x] != 0, qs[threadIdx.x], x1)));
}
extern "C" __global__ void p_quad_step_of(fe* o, const fe* p, const fe* qs, const int* u) {
    const fe x = p[threadIdx.x];
    o[threadIdx.x] = quad_of_next(ge_quad_of_step(x, fe_sel(u[threadIdx.x] != 0, qs[threadIdx.x], x)));
}
extern "C" __global__ void p_pair_step_of(fe* o, const fe* p, const fe* qs, const int* u) {
    const fe oa = p[2 * threadIdx.x], ob = p[2 * threadIdx.x + 1];
    const bool ad = u[threadIdx.x] != 0;
    fe r1, r2;
    ge_pair_of_step(oa, ob, fe_sel(ad, qs[2 * threadIdx.x], oa), fe_sel(ad, qs[2 * threadIdx.x + 1], ob), r1, r2);
    const bool odd = threadIdx.x & 1;
    const fe snd = fe_sel(odd, r2, r1), got = fe_pair_swap(snd);
    fe sm, df;
    fe_addsub(got, snd, sm, df);
    o[2 * threadIdx.x] = fe_sel(odd, sm, df);
    o[2 * threadIdx.x + 1] = fe_sel(odd, r1, r2);
}
extern "C" __global__ void p_quad_dbl_of(fe* o, const fe* p) {
    const fe x = p[threadIdx.x];
    o[threadIdx.x] = quad_of_next(ge_quad_of_step<true>(x, x));
}
extern "C" __global__ void p_row_step_of(fe* o, const fe* p, const fe* qs, const int* u) {
    const fe x = p[threadIdx.x];
    o[threadIdx.x] = row_of_next(ge_row_of_step(x, fe_sel(u[threadIdx.x] != 0, qs[threadIdx.x], x)));
}
// the whole per-lane scalar-mult loop (the k_terms<1> hot loop): tools/isa_count.py --loop prints
// the instructions of its loop body (one unified step + the bit bookkeeping)
extern "C" __global__ void p_sm_lane_zone(ge* o, const fe* s, const ge* p, const ge* dtab) {
    __shared__ geq qs[256];
    qs[threadIdx.x] = ge_prep(p[threadIdx.x]);
    o[threadIdx.x] = sm_lane_loop<true, true>(s[threadIdx.x], &qs[threadIdx.x], dtab, nullptr, 0);
}
