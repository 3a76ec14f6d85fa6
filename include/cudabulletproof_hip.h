/* cudabulletproof_hip.h — C ABI of libcudabulletproof_hip.so (MI355X / gfx950).
 *
 * Part 1 is the drop-in boundary: every entry point of the reference's
 * cuda_bulletproof.h, same names, same argument meaning, same conventions
 * (host pointers owned by the caller, synchronous, inputs never modified,
 * length mismatch -> message on stderr and *result untouched / false,
 * device errors -> message on stderr and exit(EXIT_FAILURE), as CUDA_CHECK does
 * in cuda_bulletproof_kernels.cu:13-21).  The reference's bulletproof_range_proof.cu
 * and complete_bulletproof_test.cu link against this library unchanged
 * (INTEGRATION.md).
 *
 * Part 2 is additive: batched, device-resident entry points (flat wire format,
 * explicit stream, error codes) used by the Python package and bench.py.  Every
 * `void* stream` is a hipStream_t; NULL means the default (null) stream.
 *
 * The types are layout-identical to the reference's (curve25519_ops.h:15-25,
 * bulletproof_vectors.h:8-17, :65-74, bulletproof_range_proof.h:7-18); when the
 * reference headers are included first, theirs are used.
 */
#ifndef CUDABULLETPROOF_HIP_H
#define CUDABULLETPROOF_HIP_H

#include <stddef.h>
#include <stdint.h>
#ifndef __cplusplus
#include <stdbool.h>
#endif

#ifndef CURVE25519_OPS_H
typedef struct { uint64_t limbs[4]; } fe25519;              /* curve25519_ops.h:15-17 */
typedef struct { fe25519 X, Y, Z, T; } ge25519;              /* curve25519_ops.h:20-25 */
#endif
#ifndef BULLETPROOF_VECTORS_H
typedef struct { fe25519* elements; size_t length; } FieldVector;   /* bulletproof_vectors.h:8-11 */
typedef struct { ge25519* elements; size_t length; } PointVector;   /* bulletproof_vectors.h:14-17 */
typedef struct {                                                    /* bulletproof_vectors.h:65-74 */
    size_t n;
    FieldVector a;
    FieldVector b;
    fe25519 c;
    PointVector L;
    PointVector R;
    size_t L_len;
    fe25519 x;
} InnerProductProof;
#endif
#ifndef BULLETPROOF_RANGE_PROOF_H
typedef struct {                                                    /* bulletproof_range_proof.h:7-18 */
    ge25519 V, A, S, T1, T2;
    fe25519 taux, mu, t;
    InnerProductProof ip_proof;
} RangeProof;
#endif

#ifdef __cplusplus
extern "C" {
#endif

/* ===================================================================== Part 1: reference surface */

/* cuda_bulletproof.h:13 (cuda_bulletproof_kernels.cu:62). result = canonical-tree sum of
 * device-normalized scalar*point terms. */
void cuda_point_vector_multi_scalar_mul(ge25519* result, const FieldVector* scalars, const PointVector* points);
/* cuda_bulletproof.h:17 (cuda_bulletproof_kernels.cu:119): same result. */
void cuda_point_vector_multi_scalar_mul_shared(ge25519* result, const FieldVector* scalars,
                                               const PointVector* points);

/* cuda_bulletproof.h:22 (cuda_inner_product.cu:97): the reference's GPU reduction order
 * (n <= 512: block halving tree; n > 512: grid-stride + two trees). */
void cuda_field_vector_inner_product(fe25519* result, const FieldVector* a, const FieldVector* b);
/* cuda_bulletproof.h:26 (declared there, never defined with C linkage in the reference):
 * the n <= 512 halving-tree order for any n. */
void cuda_field_vector_inner_product_shared(fe25519* result, const FieldVector* a, const FieldVector* b);
/* cuda_inner_product.cu:302 (extern "C", not in the reference header). */
void cuda_batch_field_vector_inner_product(fe25519* results, const FieldVector* a_vectors,
                                           const FieldVector* b_vectors, size_t num_vectors);

/* cuda_bulletproof.h:31-46 (cuda_field_ops.cu:257, :293, :329, :374). */
void cuda_batch_field_add(fe25519* results, const fe25519* a, const fe25519* b, size_t count);
void cuda_batch_field_sub(fe25519* results, const fe25519* a, const fe25519* b, size_t count);
void cuda_batch_field_mul(fe25519* results, const fe25519* a, const fe25519* b, size_t count);
void cuda_batch_field_mul_karatsuba(fe25519* results, const fe25519* a, const fe25519* b, size_t count);
/* reproduces field_square_kernel (cuda_field_ops.cu:147), which is NOT fe25519_sq */
void cuda_batch_field_square(fe25519* results, const fe25519* inputs, size_t count);
/* cuda_bulletproof.h:50 (cuda_field_ops.cu:405): the reference kernel races;
 * this defines it as the host fe25519_invert chain applied elementwise. */
void cuda_batch_field_invert(fe25519* results, const fe25519* inputs, size_t count);
/* cuda_bulletproof.h:55 (cuda_field_ops.cu:533): limbwise u64 add, no carry, no reduction */
void cuda_soa_field_add(fe25519* results, const fe25519* a, const fe25519* b, size_t count);

/* cuda_bulletproof.h:61 (cuda_range_proof_verify.cu:82, notebook-only in the reference). */
bool cuda_range_proof_verify(const RangeProof* proof, const ge25519* V, size_t n, const PointVector* G,
                             const PointVector* H, const ge25519* g, const ge25519* h);
/* cuda_bulletproof.h:72 (cuda_range_proof_verify.cu:130). */
bool cuda_inner_product_verify(const InnerProductProof* proof, const ge25519* P, const PointVector* G,
                               const PointVector* H, const ge25519* Q);

/* cuda_bulletproof.h:81-84: declared but never defined by the reference; here they time the
 * corresponding GPU path and print one line each. */
void cuda_benchmark_multi_scalar_mul(int iterations, size_t vector_size);
void cuda_benchmark_inner_product(int iterations, size_t vector_size);
void cuda_benchmark_field_operations(int iterations, size_t batch_size);
void cuda_benchmark_range_proof(int iterations, size_t bit_size);

/* ===================================================================== Part 2: batched device API */

/* Flat wire format of a batch of range proofs; every pointer is DEVICE memory.
 * Per proof p: V[p], A[p], S[p], T1[p], T2[p], t[p], c[p], x[p]; a/b: ab_len entries
 * at p*ab_len; L/R: L_len entries at p*L_len (L[0]/R[0] are never read, crv:180-205).
 * V is the caller's V argument of the verify.  taux, mu and Vp (the proof's own V) are read
 * only by the range_proof_verify semantics (hipbp_batch_range_proof_verify_std); Vp NULL means
 * "equal to V". */
typedef struct {
    size_t count, n, ab_len, L_len;
    const ge25519 *V, *A, *S, *T1, *T2;
    const fe25519 *t, *a, *b, *c, *x;
    const ge25519 *L, *R;
    const fe25519 *taux, *mu;
    const ge25519* Vp;
} hipbp_proof_batch;

typedef enum {
    HIPBP_OK = 0,
    HIPBP_ERR_ARG = 1,       /* unsupported shape / null pointer */
    HIPBP_ERR_DEVICE = 2,    /* HIP runtime error (message via hipbp_last_error) */
} hipbp_status;

const char* hipbp_last_error(void);
/* Number of HIP devices visible. */
int hipbp_device_count(void);

/* cuda_range_proof_verify (cuda_bulletproof.h:61, crv:82) over an ARRAY of the reference's own host
 * structs: ok[i] = cuda_range_proof_verify(&proofs[i], &V[i], n, G, H, g, h) for i < count, bit for
 * bit, with the reference's length check per proof (message on stderr, ok[i] = 0).  The proofs are
 * packed into the flat batch format, sharded in contiguous blocks over num_gpus devices (<= 0: all
 * visible; more than are visible: HIPBP_ERR_ARG, nothing verified) starting at the calling thread's
 * current device (shard d on device (current + d) mod the device count, so num_gpus = 1 stays on
 * the current device), one host thread per device: 1024-proof chunks are packed into pinned staging, copied
 * and pushed as they are packed, alternating over two verify pipelines on two streams; one D2H of
 * the verdicts; no data-path exchange between devices.  Each device's engine keeps the fixed-base
 * prefix tables of the last generator set it was called with (G | H | h, exact byte compare;
 * HIPBP_HOST_PREFIX_BITS, default 16, at most 1.25 GB; 0: none), so calls after the first against
 * the same generators run the table-started scalar multiplications.  Proofs whose a/b length or round
 * count differs from the first valid proof's go through the single-proof path.  Host pointers,
 * synchronous.  Returns HIPBP_OK or an error code (hipbp_last_error); on an error ok is
 * undefined.  No reference counterpart (the additive batch entry point). */
int hipbp_batch_range_proof_verify_host(const RangeProof* proofs, const ge25519* V, size_t count, size_t n,
                                        const PointVector* G, const PointVector* H, const ge25519* g,
                                        const ge25519* h, int num_gpus, uint8_t* ok);

/* Batched cuda_range_proof_verify semantics. G/H: n generators, g/h: 1 point (device).
 * ok[count] gets 1/0; P_out / check_out (nullable) get the IPA point P and the check point. */
int hipbp_batch_range_proof_verify(const hipbp_proof_batch* batch, const ge25519* G, const ge25519* H,
                                   const ge25519* g, const ge25519* h, uint8_t* ok, ge25519* P_out,
                                   ge25519* check_out, void* stream);
/* Batched range_proof_verify semantics (bulletproof_range_proof.cu:1717, the reference's CPU
 * "STANDARD VERIFICATION": V match, compute_precise_delta, enhanced_range_check,
 * robust_polynomial_identity_check, calculate_inner_product_point, inner_product_verify with its
 * own accept rule).  Needs batch->taux/mu.  Nullable extra outputs:
 * flags_out[count]: bit0 V match, bit1 enhanced_range_check, bit2 polynomial identity methods 1|2,
 * bit3 method 3, bit4 method 4, bit5 inner_product_verify;
 * poly_out[4*count]: per proof left side, right side, and the two method-3 products. */
int hipbp_batch_range_proof_verify_std(const hipbp_proof_batch* batch, const ge25519* G, const ge25519* H,
                                       const ge25519* g, const ge25519* h, uint8_t* ok, ge25519* P_out,
                                       ge25519* check_out, uint8_t* flags_out, ge25519* poly_out, void* stream);
/* Batched cuda_inner_product_verify semantics; P[count] given (device). */
int hipbp_batch_inner_product_verify(const hipbp_proof_batch* batch, const ge25519* P, const ge25519* G,
                                     const ge25519* H, const ge25519* Q, uint8_t* ok, ge25519* check_out,
                                     void* stream);
/* Streaming verify pipeline.  A verify has a log2(n)+1-deep chain of dependent stages
 * (stage 0, IPA fold rounds 1..L-1, final); the pipeline keeps up to log2(n)+1 batches in
 * flight and each push runs ONE tick: stage 0 of the pushed batch, round r of the batch
 * pushed r ticks earlier, the final stage of the oldest, all in one kernel launch.
 * A batch's outputs (ok / P_out / check_out, device memory) are complete after
 * depth-1 further pushes or a flush; its inputs (and P_in) are consumed by its own push.
 * range_mode 1: cuda_range_proof_verify semantics (h = the generator h; g may be NULL);
 * range_mode 2: range_proof_verify semantics (g, h the generators; batch taux/mu required);
 * range_mode 0: cuda_inner_product_verify semantics (h = Q, P_in required, g may be NULL).
 * Returns NULL on error (see hipbp_last_error). */
void* hipbp_pipeline_create(size_t max_batch, size_t n, int range_mode, const ge25519* G, const ge25519* H,
                            const ge25519* g, const ge25519* h, void* stream);
int hipbp_pipeline_push(void* pipeline, const hipbp_proof_batch* batch /* NULL = drain tick */,
                        const ge25519* P_in, uint8_t* ok, ge25519* P_out, ge25519* check_out,
                        uint8_t* flags_out /* range_mode 2, nullable */, ge25519* poly_out /* idem */);
int hipbp_pipeline_flush(void* pipeline);
int hipbp_pipeline_depth(void* pipeline);
/* Fixed-base prefix tables for the pipeline's generators (no reference counterpart; an
 * additive speed-up with the same bits).  bits = K in 1..24 builds, for each of the 2n + 2
 * bases G_i, H_i, h, g, the state of ge25519_scalarmult after every possible top-K-bit prefix
 * of a scalar ((2n + 2) * 2^K * 128 bytes of device memory: 17.4 GB at n = 64, K = 20).  The
 * scalar multiplications on those bases (the two MSMs, fold round 0, t*h, c*Q, the polynomial
 * terms on g and h) then start at bit 255 - K from the table entry; the operations after it are
 * unchanged, so every output has the same bits.  Built from the generator CONTENTS at this call
 * (synchronous); the caller must not change G/H/g/h afterwards while tables are on.  bits = 0
 * frees them.  The pipeline must be idle (flushed). */
int hipbp_pipeline_prefix_tables(void* pipeline, int bits);
/* Generator sets (no reference counterpart): a device snapshot of G[n], H[n], g, h (device
 * buffers, copied at create; the caller may free them afterwards) plus, for prefix_bits in 1..24,
 * their fixed-base prefix tables (as hipbp_pipeline_prefix_tables; 0 = none).  Synchronous.
 * Returns NULL on error.  One set serves the prover and any number of verify pipelines. */
void* hipbp_gens_create(size_t n, const ge25519* G, const ge25519* H, const ge25519* g, const ge25519* h,
                        int prefix_bits, void* stream);
void hipbp_gens_destroy(void* gens);
/* The pipeline reads its generators and prefix tables from `gens` (same n; the pipeline must be
 * idle; the set must outlive the pipeline's use of it).  Results keep their bits. */
int hipbp_pipeline_use_gens(void* pipeline, void* gens);
/* hipbp_batch_range_proof_verify with the generators and prefix tables of a generator set (same n,
 * same device): a one-shot batch that starts its generator-based scalar multiplications from the
 * tables (the pipeline path's speed without a pipeline handle).  Same bits as the plain call. */
int hipbp_batch_range_proof_verify_gens(const hipbp_proof_batch* batch, void* gens, uint8_t* ok, ge25519* P_out,
                                        ge25519* check_out, void* stream);
/* Split stage 0 for the batches pushed from now on (on = 1; range_mode 1 or 2, 4 <= n <= 64): a
 * batch's stage-0 tick runs only fold round 0 (and the range_proof_verify polynomial terms); its
 * two MSMs' terms, t*h and c*Q, which only the final assembly reads, run in chunks inside its
 * fold-round ticks, whose own items shrink round by round.  A finite batch then fills the rounds
 * before its latency-bound last ticks.  Same bits either way.  HIPBP_ERR_ARG where it does not
 * apply: inner-product mode, n above the lane-tree limit (HIPBP_LANE_TREE_MAX), or n > 512 (a
 * split tick's 2 log2 n + 5 regions must fit the kernel's region list). */
int hipbp_pipeline_defer_msm(void* pipeline, int on);
void hipbp_pipeline_destroy(void* pipeline);

/* ---- prover: generate_range_proof (bulletproof_range_proof.cu:1159) + inner_product_prove
 * (bulletproof_vectors.cu:277) + fix_inner_product_proof (rp.cu:198), batched, bit-exact.
 * The prover's randomness is an input: each random scalar is the 32 bytes that
 * generate_random_scalar (rp.cu:153) produces (RAND_bytes + its masks), as 4 LE limbs.
 * All pointers DEVICE memory.  n: power of two, 1..128 (validate_range_input reads byte n/8). */
typedef struct {
    size_t count, n;
    const fe25519* v;       /* [count] value (fe25519_frombytes of the value bytes) */
    const fe25519* gamma;   /* [count] blinding of V = g^v h^gamma */
    const fe25519* sL;      /* [count*n] */
    const fe25519* sR;      /* [count*n] */
    const fe25519* rnd;     /* [count*4] alpha, rho, tau1, tau2 */
} hipbp_prove_input;
/* Output in the flat wire format of hipbp_proof_batch (ab_len = 1, L_len = log2 n), so it can be
 * verified as is.  valid[p] = 0: validate_range_input refused the value; the proof is then the
 * reference's zeroed one (V, A, S, T1, T2 identity; taux, mu, t 0; the rest 0). */
typedef struct {
    ge25519 *V, *A, *S, *T1, *T2;          /* [count] */
    fe25519 *taux, *mu, *t, *c, *x;        /* [count] */
    fe25519 *a, *b;                        /* [count] */
    ge25519 *L, *R;                        /* [count*L_len] */
    uint8_t* valid;                        /* [count] */
} hipbp_proof_out;
int hipbp_batch_generate_range_proof(const hipbp_prove_input* in, const ge25519* G, const ge25519* H,
                                     const ge25519* g, const ge25519* h, hipbp_proof_out* out, void* stream);
/* The same with a generator set's generators and prefix tables (every scalar multiplication of
 * the prover is on G_i, H_i, g or h); same bits as hipbp_batch_generate_range_proof on them. */
int hipbp_batch_generate_range_proof_gens(const hipbp_prove_input* in, void* gens, hipbp_proof_out* out,
                                          void* stream);

/* Canonical-tree MSM on device buffers.  Asynchronous on `stream`; the MSM, MSM-batch
 * and point-tree calls keep one workspace per (device, stream), so calls on different streams may
 * run concurrently. */
int hipbp_msm(ge25519* result, const fe25519* scalars, const ge25519* points, size_t n, void* stream);

/* count independent canonical-tree MSMs of n points each over the SAME points (e.g. the IPA
 * commitments P = MSM(a||b, G||H) of a batch of proofs): scalars
 * [count*n] (MSM k = rows k*n .. k*n+n-1), points [n], results [count]; each result is bit-exact
 * with hipbp_msm on its rows.  Device buffers. */
int hipbp_msm_batch(ge25519* results, const fe25519* scalars, const ge25519* points, size_t n, size_t count,
                    void* stream);

/* hipbp_msm_batch over a generator set's G||H (2n points, hipbp_gens_create) with its fixed-base
 * prefix tables: each point's scalar multiplication starts from the table entry of its scalar's
 * top K bits, so every result has hipbp_msm_batch's bits with fewer point operations.  scalars
 * [count*2n] (MSM k = rows k*2n .. k*2n+2n-1, the a||b of an IPA commitment P), results [count]. */
int hipbp_msm_batch_gens(ge25519* results, const fe25519* scalars, const void* gens, size_t count, void* stream);

/* Pippenger bucket MSM with window_bits-bit windows (4..12; BASELINE configs[2] names 12), over
 * the same fe25519/ge25519 arithmetic, on device buffers.  A LABELLED ALTERNATIVE, not a drop-in
 * for cuda_point_vector_multi_scalar_mul: the reference's MSM bits come from per-point
 * double-and-add + the canonical tree (hipbp_msm), and this arithmetic is not associative, so a
 * bucket regrouping yields different bits.  Its own result is fixed (stable bucket order, fixed
 * trees) and equals the C restatement oracle/bp_oracle.c orc_msm_pippenger.  Asynchronous: the
 * host does not wait (the bucket-tree depth is read on the device); the Horner chain runs on an
 * internal side stream that the caller's stream waits on, so the result is ready in the caller's
 * stream order.  Workspaces are per (device, stream): MSMs on different streams run concurrently.
 * No reference counterpart. */
int hipbp_msm_pippenger(ge25519* result, const fe25519* scalars, const ge25519* points, size_t n,
                        int window_bits, void* stream);
/* count Pippenger MSMs over the SAME n device points in one call: results[m] = hipbp_msm_pippenger
 * of scalars[m n .. m n + n) (bit for bit).  One sort, one set of bucket-tree launches and one
 * Horner launch serve all of them, so the latency-bound chains are shared.  count <= 65535. */
int hipbp_msm_pippenger_batch(ge25519* results, const fe25519* scalars, const ge25519* points, size_t n,
                              size_t count, int window_bits, void* stream);
/* The two halves of hipbp_msm_pippenger, for a multi-GPU MSM that splits the windows over the
 * ranks (cudabulletproof_amd/shard.py sharded_msm_pippenger).  _windows writes the
 * window sums S_w, w in [w_begin, w_end), into window_sums[w] (W = ceil(256 / window_bits)
 * entries; the others are left untouched), each with the bits the single call forms; _horner
 * runs the Horner chain over all W sums of each of count MSMs (window_sums[m W .. m W + W)), so
 * every rank that holds all sums gets hipbp_msm_pippenger's result bit for bit.  Device buffers,
 * asynchronous on `stream`. */
int hipbp_msm_pippenger_windows(ge25519* window_sums, const fe25519* scalars, const ge25519* points, size_t n,
                                int window_bits, int w_begin, int w_end, void* stream);
int hipbp_msm_pippenger_horner(ge25519* results, const ge25519* window_sums, size_t count, int window_bits,
                               void* stream);
/* Canonical tree over n device points: for stride 1, 2, 4, ...: T[i] = Ndev(T[i] + T[i+stride])
 * for i % (2 stride) == 0 and i + stride < n; result = T[0] (the reduction half of
 * cuda_bulletproof_kernels.cu:45-115).  hipbp_msm = this tree over the per-point
 * terms; a multi-GPU MSM combines per-rank shard roots with it. */
int hipbp_point_tree(ge25519* result, const ge25519* points, size_t n, void* stream);
/* Elementwise device field ops: op 0 add, 1 sub, 2 mul, 3 square (reference kernel quirk),
 * 4 SoA add (limbwise, no carry), 5 invert (host chain), 6 the product fold alone on the
 * 512-bit t = a || b (fe25519_mul's reduction, curve25519_ops.cu:114-145), 7 fe25519_sq,
 * 8 / 9 the sum / difference of the fused add-and-sub block the lane-quad forms use (the same
 * values as ops 0 / 1), 10 fe25519_mul formed as the drain forms' quad-split product (fe_mul_q4:
 * four lanes per element, the same value as op 2), 11 fe25519_mul(a, k) for the curve constant k
 * (fe_mul_k: only provably possible carries counted; the same value as op 2 with b = k; b unused),
 * 12 the same split over a lane quad (fe_mul_q4_k, four lanes per element); the 16-lane row step's
 * field blocks (same values as ops 0 / 8 / 9 / 6): 13 add, 15 / 16 add-sub, 19 fold in their latency
 * forms, and 14, 17 / 18, 20 the same through their deferred rare-edge test (fast form, recomputed
 * when the element's test words hit 2^32-1). */
int hipbp_field_op(int op, fe25519* r, const fe25519* a, const fe25519* b, size_t count, void* stream);
/* The verify path's SHA-256 message shapes on the device, item i over in[6i .. 6i+5] (device
 * pointers): kind 0 the y challenge (points (in0,in1), (in2,in3), (in4,in5) as X, Y), 1 z (in0),
 * 2 x (points (in0,in1), (in2,in3)), 3 an inner-product round challenge (transcript in0, L.X in1,
 * R.X in2), 4 the prover's IPA transcript start (t in0, taux in1, mu in2), 5 the unmasked digest of
 * in0..in3 in raw limb order.  For checking against FIPS 180-4 (bulletproof_challenge.cu:6-77). */
int hipbp_sha_probe(int kind, fe25519* out, const fe25519* in, size_t count, void* stream);
/* Frees every workspace the library caches for `stream` on the current device (canonical MSM /
 * point-tree, prover, one-shot verify pipelines, the Pippenger workspace pair with its side stream
 * and events), after waiting for the stream.  Workspaces otherwise live as long as the process;
 * a caller that makes short-lived streams calls this before destroying one.  No reference
 * counterpart. */
int hipbp_release_stream_workspaces(void* stream);
/* Wait for `stream`. */
int hipbp_sync(void* stream);

/* Per-kernel HIP-event timing of the verify pipeline (on the stream the kernels run on).
 * enable(1) resets the accumulators; collect() waits for the recorded events and returns,
 * per kernel kind, the summed launch durations (ms) and the launch counts. */
int hipbp_timing_enable(int on);
int hipbp_timing_collect(double* total_ms, uint64_t* launches);
int hipbp_kernel_count(void);
const char* hipbp_kernel_name(int kind);

#ifdef __cplusplus
}
#endif
#endif
