// bp_kernels.h — host-side launch interface of the gfx950 kernels (internal to the library).
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

namespace bp {
struct fe;
struct ge;

// Device view of a batch of range proofs in the flat wire format (include/cudabulletproof_hip.h).
struct BatchView {
    int B;        // proofs
    int n;        // range bits = generator count (power of two)
    int ab_len;   // length of the proof's a/b vectors (>= 1)
    int L_len;    // IPA rounds (log2 n)
    const ge* V;  // [B] value commitments (the V argument of cuda_range_proof_verify)
    const ge* A;  // [B]
    const ge* S;  // [B]
    const ge* T1; // [B]
    const ge* T2; // [B]
    const fe* t;  // [B]
    const fe* a;  // [B*ab_len]
    const fe* b;  // [B*ab_len]
    const fe* c;  // [B]
    const fe* x;  // [B]
    const ge* L;  // [B*L_len]
    const ge* R;  // [B*L_len]
    const fe* taux;   // [B]  range_proof_verify semantics only
    const fe* mu;     // [B]
    const ge* Vp;     // [B]  the proof's own V (== V when the caller passed none)
};

// Device workspace of one verify batch (allocated by the engine).
struct VerifyWs {
    fe* sG;        // [B]      MSM scalar for G (raw limbs)
    fe* sH;        // [B*n]    MSM scalars for H (raw limbs)
    fe* sc;        // [B*4]    canonical t, a0, b0, c
    fe* u;         // [B*L_len] canonical u_r
    fe* uinv;      // [B*L_len] canonical "u_r^-1"
    uint8_t* ipok; // [B]
    ge* msm_pts;   // [B*2*n]  per-point MSM terms
    ge* msm_part;  // [B*2]    tree results: <sG,G>, <sH,H>
    ge* terms;     // [B*4]    slots 2,3: t*h, c*Q
    ge* fold[2];   // [B*2n]   per-round scalar-mult terms, round r in fold[r & 1]; the next round's
                   //          tasks combine them into the folded G'/H' they consume (crv:230, :240)
    ge* fin;       // [B*2]    a0*G', b0*H'
    ge* Pin;       // [B]      given P (inner-product-only verify)
    // range_proof_verify semantics (mode 2) only:
    fe* psc;       // [B*8]    canonical t, taux, z^2, delta, mu, x, x^2 (polynomial identity scalars)
    ge* pterm;     // [B*8]    g^t, h^taux, V^z^2, g^delta, h^mu, T1^x, T2^x^2 (host-normalized)
    ge* lr;        // [B*2]    left / right side of the polynomial identity
    fe* chal;      // [B]      SHA-256 of the sides' bytes (method 3 scalar, raw bytes)
    ge* m3;        // [B*2]    chal * left, chal * right
    uint8_t* rflags;   // [B]  bit0 V match, bit1 range check, bit2 methods 1|2
    ge* pbase;     // [B*3]    V, T1, T2 copied by the prep task: stage 0 runs a tick after the push and
               //          must not read the caller's batch (consumed by its own push)
};

// One batch in flight in the verify pipeline (device-resident copy, read by the tick kernels).
struct SlotDev {
    BatchView bv;
    VerifyWs ws;
    uint8_t* ok;
    ge* P_out;
    ge* chk_out;
    uint8_t* flags_out;   // mode 2, nullable
    ge* poly_out;         // mode 2, nullable
    int range_mode;       // 0 inner product only, 1 cuda_range_proof_verify, 2 range_proof_verify
    int lane_tree;        // MSM trees reduced by final_task's lane (n <= lane-tree limit), else RK_TREE
    // Lane orders of the per-lane-scalar item sets (nullable = index order), written by
    // launch_lane_sort after the batch's challenge tick: the lanes of a wave take items of equal
    // scalar-mult chain length.  perm0: stage-0 per-lane items; permr[r]: fold round r; perm_ft:
    // the final terms.
    uint32_t* perm0;
    uint32_t* permr[17];
    uint32_t* perm_ft;
    // Fixed-base prefix tables of the pipeline's generators (nullable; ge25519_dev.h): base b's
    // table is ptab[b << pbits ..], b = k for G_k, n + k for H_k, 2n for h (= Q), 2n + 1 for g.
    const ge* ptab;
    int pbits;
    // 1: stage 0 is split (Pipeline "deferred MSM terms"): RK_STAGE0 runs only the items later
    // stages wait for (fold round 0, mode-2 polynomial terms); the two MSMs' terms and t*h, c*Q,
    // which only the lane trees and the final assembly read, run as RK_MSMT chunks in the fold ticks
    int defer;
};

// Stage-0 lane layout (host and device).  stage0_task's items by class — the <sG,G>/<sH,H>
// terms, IPA fold round 0, t*h / c*Q, the 7 polynomial terms: each class is one call site of
// the scalar multiplication, so a wave must not mix classes.  For n >= 64 the scalar-uniform
// items come first (U lanes: the <sG,G> segments, one scalar per n items, then fold round 0, one
// scalar per n-item half); then the per-lane classes, each in its own wave-aligned lane range
// (sorted by chain length when SlotDev::perm0 is set): [<sH,H> (n < 64: all MSM terms)]
// [fold round 0 (n < 64 only)] [t*h, c*Q] [poly terms].
struct Stage0Lanes {
    unsigned long long U;
    unsigned long long off[4], size[4];   // lane offset / items of each per-lane class
    unsigned long long total;             // region lanes
    unsigned long long pl;                // per-lane items (perm0 length)
};
// sel: S0_ALL every stage-0 item; S0_CRIT the split stage 0's RK_STAGE0 part (fold round 0 and
// the polynomial terms); S0_DEFER its RK_MSMT part (the MSM terms, t*h and c*Q).  The per-lane
// classes keep their S0_ALL positions in perm0 (the lane sort always orders all of them).
enum Stage0Sel { S0_ALL = 0, S0_CRIT = 1, S0_DEFER = 2 };
__host__ __device__ inline Stage0Lanes stage0_lanes(unsigned long long B, int n, int L, int range_mode, int sel = S0_ALL) {
    Stage0Lanes z;
    const unsigned long long msm = range_mode ? B * 2 * n : 0, fold = L > 0 ? B * 2 * n : 0;
    const bool uni = n >= 64;
    const bool m = sel != S0_CRIT, f = sel != S0_DEFER;   // MSM-side / fold-side items included
    z.U = uni ? (m ? msm / 2 : 0) + (f ? fold : 0) : 0;
    z.size[0] = m ? (uni ? msm / 2 : msm) : 0;
    z.size[1] = f && !uni ? fold : 0;
    z.size[2] = m ? B * 2 : 0;
    z.size[3] = f && range_mode == 2 ? B * 7 : 0;
    unsigned long long o = z.U, pl = 0;
    for (int c = 0; c < 4; c++) {
        z.off[c] = o;
        o += (z.size[c] + 63) & ~63ull;
        pl += z.size[c];
    }
    z.total = o;
    z.pl = pl;
    return z;
}
// log2 of a power of two (host and device)
__host__ __device__ inline int log2n(int n) { return __builtin_ctz((unsigned)n); }

// Per-lane class c item j -> stage0_task's item index (perm0 holds, per class range, the
// items of that class in chain-length order: perm0[pl_base(c) + j]).
__host__ __device__ inline uint32_t stage0_class_item(const SlotDev& sd, int c, uint32_t j) {
    const uint32_t B = (uint32_t)sd.bv.B;
    const int n = sd.bv.n, ln = log2n(n);
    const uint32_t nA = sd.range_mode ? B << (ln + 1) : 0, nB = sd.bv.L_len > 0 ? B << (ln + 1) : 0;
    if (c == 0) return n >= 64 ? ((j >> ln) << (ln + 1)) + n + (j & (n - 1)) : j;
    if (c == 1) return nA + j;
    if (c == 2) return nA + nB + j;
    return nA + nB + 2 * B + j;
}

// Stage-0 lane -> stage0_task item, or SIZE_MAX for a padding lane (stage0_lanes; sel: the
// part of a split stage 0 the region runs, Stage0Sel).
__host__ __device__ inline uint32_t stage0_item(const SlotDev& sd, uint32_t l, int sel = S0_ALL) {
    const uint32_t B = (uint32_t)sd.bv.B;
    const int n = sd.bv.n, ln = log2n(n);
    const Stage0Lanes z = stage0_lanes(B, n, sd.bv.L_len, sd.range_mode, sel);
    if (l < (uint32_t)z.U) {
        const uint32_t nG = (sd.range_mode && sel != S0_CRIT) ? B << ln : 0;
        if (l < nG) return ((l >> ln) << (ln + 1)) + (l & (n - 1));   // <sG,G> segment of proof l / n
        return (sd.range_mode ? B << (ln + 1) : 0) + (l - nG);
    }
    const Stage0Lanes za = sel == S0_ALL ? z : stage0_lanes(B, n, sd.bv.L_len, sd.range_mode);
    int c = 0;
    uint32_t base = 0;   // class c's offset in perm0 (the S0_ALL class sizes)
#pragma unroll
    for (int k = 1; k < 4; k++)
        if (l >= (uint32_t)z.off[k]) { c = k; base += (uint32_t)za.size[k - 1]; }
    const uint32_t j = l - (uint32_t)z.off[c];
    if (j >= (uint32_t)z.size[c]) return UINT32_MAX;
    return stage0_class_item(sd, c, sd.perm0 ? sd.perm0[base + j] : j);
}

// Fold round r >= 1 runs per-lane scalars when a scalar's 2n' items are fewer than a wave.
__host__ __device__ inline bool round_per_lane(int n, int r) { return (n >> r) < 64; }

// Counting sort of one batch's per-lane item sets by chain length (see SlotDev::perm0).
constexpr int MSM_BINS = 513;   // chain lengths 0..512

enum SortSetKind { SS_STAGE0 = 0, SS_ROUND = 1, SS_FT = 2 };
constexpr int LANE_SORT_SETS = 18;
constexpr int LANE_SORT_BLOCK = 256;   // one wave per SIMD: fits beside a running k_terms launch
struct LaneSortPlan {
    int count;
    int pad;
    const SlotDev* slot;   // device copy of the batch's slot
    struct Set {
        int kind, r;
        unsigned long long items;
        uint32_t* perm;
        unsigned block0;   // first block of this set in the hist / scatter grids
        unsigned pad;
    } set[LANE_SORT_SETS];
    unsigned blocks;
    int longest_first;
};
void launch_lane_sort(const LaneSortPlan& plan, unsigned* bins, unsigned* offs, hipStream_t s);

// A tick's work list (one k_terms launch): region k covers items [begin_k, begin_{k+1}) of one
// slot at one stage.  RK_TREE (block-level MSM tree; always first, 256-aligned), RK_PREP
// (challenges/scalars, one lane per proof and kind), RK_STAGE0, RK_ROUND, RK_FINAL_TERMS,
// RK_POLY (mode 2: polynomial identity sides), RK_M3 (mode 2: method-3 products), RK_FINAL
// (P, check point, accept).
enum RegionKind { RK_STAGE0 = 0, RK_ROUND = 1, RK_FINAL_TERMS = 2, RK_FINAL = 4, RK_PREP = 5,
                  RK_TREE = 6, RK_POLY = 7, RK_M3 = 8,
                  RK_LTREE = 9 /* the n <= LANE_TREE_MAX MSM trees, one lane (quad) per proof, into msm_part */,
                  RK_MSMT = 10 /* a chunk of split stage 0's deferred part (SlotDev::defer); Region::r = its first lane */ };
struct Region {
    int kind;
    int slot;
    int r;
    int pad;
    unsigned long long begin;
    unsigned long long items;   // lanes [begin+items, next begin) are wave-alignment padding
};
// MSMs of at most this many points (the range proofs') are reduced by one lane per proof (the
// RK_LTREE region, a few ticks before the final one), one MSM tree per lane (63 adds for n = 64,
// lanes fully busy, latency well inside a tick);
// larger ones by RK_TREE blocks (levels 1..128 with LDS barriers) + final_task's upper levels.
constexpr int LANE_TREE_MAX = 64;
constexpr int MAX_REGIONS = 24;   // >= log2(MAX_N) + 3 stages in flight + 3 stages with 2 regions
struct RegionList {
    int count;
    int pad;
    unsigned long long total;
    Region reg[MAX_REGIONS];
};

// Kernel groups of the verify pipeline, for per-kernel HIP-event timing (bench.py roofline).
enum KernelKind { KT_PREP = 0, KT_TERMS, KT_TREE, KT_COMBINE, KT_COUNT };

// Prefix tables (SlotDev::ptab) of the bases G[0..n), H[0..n), h, g (g nullable: its rows are
// left unwritten): tab[(2n + 2) << K].
void launch_prefix_tables(ge* tab, const ge* G, const ge* H, const ge* h, const ge* g, int n, int K, hipStream_t s);
// ql: lanes per scalar-multiplication item (1; 2: lane pairs; 4: lane quads, the drain-tick form,
// whose chain regions take 4 lanes per proof too; 16: 16-lane rows, chains on quads), k_terms<ql>
void launch_terms(const RegionList& rl, const SlotDev* slots, const ge* G, const ge* H, const ge* g, const ge* h,
                  const ge* dtab, const fe* two_i, hipStream_t s, int ql = 1);
// per tick form (bp_terms1.hip, bp_terms2.hip, bp_terms4.hip, bp_terms16.hip): k_terms<1 | 2 | 4 | 16>
// dst[0..bytes) = src (device-visible pinned host memory), bytes a multiple of 16, by a kernel of the
// row-form tick's code object (bp_terms16.hip)
void launch_upload(void* dst, const void* src, size_t bytes, hipStream_t s);
#define BP_DECL_TERMS(Q)                                                                                    \
    void launch_terms##Q(const RegionList& rl, const SlotDev* slots, const ge* G, const ge* H, const ge* g,  \
                         const ge* h, const ge* dtab, const fe* two_i, hipStream_t s, unsigned lds_pad);
BP_DECL_TERMS(1)
BP_DECL_TERMS(2)
BP_DECL_TERMS(4)
BP_DECL_TERMS(16)
#undef BP_DECL_TERMS
inline bool region_is_sm(int kind) {
    return kind == RK_STAGE0 || kind == RK_ROUND || kind == RK_FINAL_TERMS || kind == RK_M3 || kind == RK_MSMT;
}
// lanes per item of a region in the form with ql lanes per scalar multiplication (the chain regions
// go on quads in the quad and row forms only)
inline int region_lanes(int kind, int ql) {
    if (region_is_sm(kind)) return ql;
    return (ql >= 4 && (kind == RK_FINAL || kind == RK_LTREE || kind == RK_PREP)) ? 4 : 1;
}

// Generic canonical-tree MSM.  perm [m] / bins [MSM_BINS] (nullable): workspace of the
// counting sort that groups items of equal chain length into the same waves (m >= MSM_SORT_MIN).
constexpr size_t MSM_SORT_MIN = 4096;
void launch_msm_points(ge* pts, const fe* scal, const ge* P, size_t m, uint32_t* perm, unsigned* bins,
                       const ge* dtab, hipStream_t s, size_t pm = 0, const ge* ptab = nullptr, int K = 0);
void launch_tree(ge* out, const ge* in, int S, size_t m, hipStream_t s);
void launch_ops_scan(unsigned* bins, int longest_first, hipStream_t s);   // bins -> start offsets
// Pippenger bucket MSM (bp_pippenger.hip; hipbp_msm_pippenger), 4 <= c <= 12
// count MSMs over the same n points: results[m] = MSM(scal[m n .. m n + n), P)
hipError_t msm_pippenger(ge* result, const fe* scal, const ge* P, size_t n, size_t count, int c, const ge* dtab,
                         hipStream_t s);
hipError_t msm_pippenger_windows(ge* Sw, const fe* scal, const ge* P, size_t n, int c, int w0, int w1,
                                 const ge* dtab, hipStream_t s);
hipError_t pippenger_horner(ge* result, const ge* Sw, size_t count, int c, hipStream_t s);
// Frees the (device, stream) Pippenger workspaces of stream s (after waiting for its work).
hipError_t pippenger_release(hipStream_t s);



// ------------------------------------------------------------------ prover (bp_prove.hip)
// Inputs of a batch of generate_range_proof calls (include/cudabulletproof_hip.h hipbp_prove_input).
struct ProveIn {
    int B, n, L;
    const fe* v;       // [B] value (fe25519_frombytes of the value bytes)
    const fe* gamma;   // [B] V blinding (raw random scalar)
    const fe* sL;      // [B*n]
    const fe* sR;      // [B*n]
    const fe* rnd;     // [B*4] alpha, rho, tau1, tau2 (raw random scalars)
};
struct ProveOut {
    ge *V, *A, *S, *T1, *T2;
    fe *taux, *mu, *t, *c, *x, *a, *b;
    ge *L, *R;          // [B*L]
    uint8_t* valid;     // [B]
};
// Prover workspace (per batch).
struct ProveWs {
    fe* ps;       // [B*4n]    MSM scalars aL | aR | sL | sR (host tobytes form)
    ge* pterm;    // [B*(4n+4)] aL_i G_i | aR_i H_i | sL_i G_i | sR_i H_i | g^v | h^gamma | h^alpha | h^rho
    ge* chain;    // [B*4]     sequential MSM accumulations (point_vector_multi_scalar_mul order)
    ge* pts;      // [B*5]     V, A, S, T1, T2
    fe* st;       // [B*8]     y, z, z^2, t0, t1, t2, t, transcript
    fe* tsc;      // [B*4]     t1, tau1, t2, tau2 (tobytes form)
    ge* tt;       // [B*4]     g^t1, h^tau1, g^t2, h^tau2
    fe* acur;     // [B*n]     IPA a (folded in place)
    fe* bcur;     // [B*n]     IPA b
    fe* iscal;    // [B*2n]    round MSM scalars a_L | b_R | a_R | b_L
    fe* csc;      // [B*2]     c_L, c_R (tobytes form)
    ge* iterm;    // [B*(2n+2)] round terms + c_L Q, c_R Q
    fe* misc;     // [B*4]     taux, mu, x
    uint8_t* valid;   // [B]
    // work lists of the term launches: item ids of the non-zero scalars, heavy (> 64 bits) at
    // list[0..), light at list[cap..); cnt[0], cnt[1] their counts (zero scalars need no launch:
    // their term is a constant, dtab[256] raw / dtab[257] normalized)
    uint32_t* list;   // [2*cap], cap = B*(4n+4)
    unsigned* cnt;    // [2]
    size_t cap;
    ge* ctab;     // [2n]      N(sm(tobytes(sub(0, 1)), H_i)) | N(sm(1, G_i)): the aR_i H_i term where
                  //           aL_i = 0 and the aL_i G_i term where aL_i = 1, once per batch
    uint32_t* slist;  // [cap]  terms0's heavy list in chain-length order (nullable: list order)
    unsigned* sbins;  // [MSM_BINS] its counting-sort bins
    // fixed-base prefix tables of G, H, h, g (nullable; the SlotDev::ptab layout): every prover
    // scalar multiplication is on one of these bases (the IPA rounds use the original G, H, Q = h)
    const ge* ptab;
    int pbits;
};
enum ProveStage { PS_PREP = 0, PS_TERMS0, PS_CHAIN0, PS_COMMIT, PS_TERMS1, PS_TX, PS_RTERMS, PS_RCHAIN, PS_ROUND,
                  PS_FINAL, PS_SORT0 /* terms0's heavy-list sort, before PS_TERMS0 */ };
void launch_prove(int stage, int r, const ProveIn& in, const ProveWs& ws, const ProveOut& out, const ge* G,
                  const ge* H, const ge* g, const ge* h, const ge* dtab, const fe* two_i, hipStream_t s);

// Elementwise field ops: op 0 add, 1 sub, 2 mul, 3 square-kernel quirk, 4 soa add (limbwise, no carry)
void launch_field_op(int op, fe* r, const fe* a, const fe* b, size_t count, hipStream_t s);
void launch_sha_probe(int kind, fe* out, const fe* in, size_t count, hipStream_t s);
void launch_ip_shared(fe* out, const fe* a, const fe* b, size_t n, hipStream_t s);
void launch_ip_grid(fe* out, fe* part, const fe* a, const fe* b, size_t n, hipStream_t s);
void launch_ip_batch(fe* out, const fe* a, const fe* b, size_t n, size_t nvec, hipStream_t s);
void launch_invert(fe* r, const fe* a, size_t count, hipStream_t s);
void launch_tree_full(ge* result, const ge* in, size_t n, ge* part0, ge* part1, hipStream_t s, int S = 1);
void launch_msm_full(ge* result, const fe* scal, const ge* P, size_t n, ge* ptsbuf, ge* part0, ge* part1,
                     uint32_t* perm, unsigned* bins, const ge* dtab, hipStream_t s, size_t count = 1,
                     const ge* ptab = nullptr, int K = 0);
}  // namespace bp
