/* bp_oracle.h — TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the reference's MSM / inner-product-argument verify path
 * (ronantakizawa/cudabulletproof).  Used only by tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg, always as the checker — never by the product
 * library (cudabulletproof_amd/), which must run its HIP kernels or fail.
 *
 * Parity: pinned against oracle/_ref/libbpref.so (the reference's own host
 * sources compiled in this container by oracle/build_ref.sh) and against the
 * golden fixtures in tests/golden/ generated from it.
 *
 * Layouts are the reference's: fe25519 = 4 little-endian u64 limbs (32 B,
 * curve25519_ops.h:15-17), ge25519 = {X,Y,Z,T} (128 B, curve25519_ops.h:20-25).
 */
#ifndef BP_ORACLE_H
#define BP_ORACLE_H
#include <stddef.h>
#include <stdint.h>

typedef struct { uint64_t v[4]; } orc_fe;
typedef struct { orc_fe X, Y, Z, T; } orc_ge;

#ifdef __cplusplus
extern "C" {
#endif

/* field (host semantics == device semantics for add/sub/mul) */
void orc_fe_add(orc_fe* h, const orc_fe* f, const orc_fe* g);
void orc_fe_sub(orc_fe* h, const orc_fe* f, const orc_fe* g);
void orc_fe_mul(orc_fe* h, const orc_fe* f, const orc_fe* g);
void orc_fe_invert(orc_fe* h, const orc_fe* f);
void orc_fe_tobytes(uint8_t* out, const orc_fe* h);         /* host: canonicalising */
void orc_fe_square_kernel(orc_fe* h, const orc_fe* f);       /* cuda_field_ops.cu:147 field_square_kernel */

/* points */
void orc_ge_zero(orc_ge* h);
void orc_ge_add(orc_ge* r, const orc_ge* p, const orc_ge* q);
void orc_ge_scalarmult(orc_ge* r, const uint8_t* scalar32, const orc_ge* p);
void orc_ge_normalize_host(orc_ge* p);
void orc_ge_normalize_dev(orc_ge* p);

/* MSM */
void orc_msm_canon(orc_ge* r, const orc_fe* s, const orc_ge* P, size_t n);   /* GPU MSM semantics (A9) */
void orc_point_tree(orc_ge* r, const orc_ge* P, size_t n);                   /* the A9 tree alone */
void orc_msm_cpu(orc_ge* r, const orc_fe* s, const orc_ge* P, size_t n);     /* vectors.cu:189 (A11) */
/* Pippenger bucket MSM over the reference's arithmetic (BASELINE configs[2]'s "window=12";
 * a labelled alternative — not the reference's MSM bits, which come from per-point
 * double-and-add + the A9 tree, and this arithmetic is not associative).  The algorithm this
 * restates exactly (hipbp_msm_pippenger): see bp_oracle.c. */
void orc_msm_pippenger(orc_ge* r, const orc_fe* s, const orc_ge* P, size_t n, int c);
void orc_pippenger_windows(orc_ge* Sw, const orc_fe* s, const orc_ge* P, size_t n, int c, int w0, int w1);
void orc_pippenger_horner(orc_ge* r, const orc_ge* Sw, int c);
void orc_inner_product(orc_fe* r, const orc_fe* a, const orc_fe* b, size_t n); /* vectors.cu:101 */
void orc_ip_gpu(orc_fe* r, const orc_fe* a, const orc_fe* b, size_t n);        /* cuda_inner_product.cu:97 */
void orc_ip_gpu_shared(orc_fe* r, const orc_fe* a, const orc_fe* b, size_t n); /* cuda_inner_product.cu:185 */
void orc_ip_gpu_batch(orc_fe* r, const orc_fe* a, const orc_fe* b, size_t n, size_t nvec); /* :302 */

/* hashing / transcript */
void orc_sha256(uint8_t out[32], const uint8_t* data, size_t len);
void orc_challenge(uint8_t out[32], const uint8_t* data, size_t len, const char* dom);
void orc_base_points(orc_ge* out, size_t n, const uint8_t seed32[32]);
void orc_gh(orc_ge* g, orc_ge* h);

/* verify path (crv:82 cuda_range_proof_verify), flat proof arrays.
 * head = {V,A,S,T1,T2 : ge; taux,mu,t,c,x : fe} (the harness' FlatHead).
 * Outputs (nullable): P (128 B), check_point (128 B),
 * Gtrace/Htrace: folded generators after each round, packed (n-1 entries each). */
typedef struct {
    orc_ge V, A, S, T1, T2;
    orc_fe taux, mu, t, c, x;
} orc_head;

int orc_cuda_range_proof_verify(const orc_head* head, const orc_ge* V, size_t n, const orc_fe* a,
                                const orc_fe* b, size_t ab_len, const orc_ge* L, const orc_ge* R,
                                size_t L_len, const orc_ge* G, const orc_ge* H, const orc_ge* g,
                                const orc_ge* h, orc_ge* P_out, orc_ge* check_out, orc_ge* Gtrace,
                                orc_ge* Htrace);

int orc_cuda_inner_product_verify(size_t n, const orc_fe* a, const orc_fe* b, size_t ab_len,
                                  const orc_fe* c, const orc_ge* L, const orc_ge* R, size_t L_len,
                                  const orc_fe* x, const orc_ge* P, const orc_ge* G, const orc_ge* H,
                                  const orc_ge* Q, orc_ge* check_out, orc_ge* Gtrace, orc_ge* Htrace);

/* range_proof_verify (bulletproof_range_proof.cu:1717): the reference's CPU verify.
 * head->V is the proof's V, V the caller's.  det (nullable) receives every intermediate. */
typedef struct {
    int vmatch, range_ok, poly_ok, poly_m1, poly_m2, poly_m3, poly_m4, ip_ok;
    orc_fe delta;
    orc_ge left, right, left_mult, right_mult, P, check;
} orc_rpv_detail;

int orc_range_proof_verify(const orc_head* head, const orc_ge* V, size_t n, const orc_fe* a, const orc_fe* b,
                           size_t ab_len, const orc_ge* L, const orc_ge* R, size_t L_len, const orc_ge* G,
                           const orc_ge* H, const orc_ge* g, const orc_ge* h, orc_rpv_detail* det);

/* generate_range_proof (bulletproof_range_proof.cu:1159-1715) + inner_product_prove
 * (bulletproof_vectors.cu:277-523) + fix_inner_product_proof (rp.cu:198), with the prover's random
 * scalars given (each the 32 bytes generate_random_scalar, rp.cu:153, produced — masks applied):
 * gamma (the V blinding), sLR[2i] = sL_i, sLR[2i+1] = sR_i (n pairs, generated interleaved),
 * rnd4 = alpha, rho, tau1, tau2.  Returns -1 when validate_range_input (rp.cu:238) refuses the
 * value (outputs untouched), else 0; a/b get the final length-1 vectors, L/R log2(n) points. */
int orc_generate_range_proof(const uint8_t value32[32], const uint8_t gamma32[32], const uint8_t* sLR,
                             const uint8_t rnd4[4][32], size_t n, const orc_ge* G, const orc_ge* H, const orc_ge* g,
                             const orc_ge* h, orc_head* head_out, orc_fe* a_out, orc_fe* b_out, orc_ge* L_out,
                             orc_ge* R_out, size_t* L_len);

#ifdef __cplusplus
}
#endif
#endif
