// bp_capi.hip — the C ABI of libcudabulletproof_hip.so (include/cudabulletproof_hip.h).
//
// Part 1 keeps the reference's cuda_bulletproof.h conventions: host buffers in, result
// out, synchronous, stderr message + early return on a length mismatch, stderr message
// + exit(EXIT_FAILURE) on a device error (CUDA_CHECK, cuda_bulletproof_kernels.cu:13-21).
// Unlike the reference it does not cudaMalloc/cudaFree per call: a per-process engine
// keeps grow-only device buffers, the identity-doubling and 2^i tables, and one stream.
#include <hip/hip_runtime.h>
#include <map>
#include <tuple>
#include <mutex>
#include <string>
#include <vector>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <algorithm>
#include <chrono>
#include <thread>

#include "../../include/cudabulletproof_hip.h"
#include "bp_kernels.h"
#include "ge25519_dev.h"

static_assert(sizeof(fe25519) == 32, "fe25519 layout");
static_assert(sizeof(ge25519) == 128, "ge25519 layout");
static_assert(sizeof(bp::fe) == 32 && sizeof(bp::ge) == 128, "device layout");
static_assert(sizeof(InnerProductProof) == 144, "InnerProductProof layout (SURVEY 8b)");
static_assert(sizeof(RangeProof) == 880, "RangeProof layout (SURVEY 8b)");

namespace {

thread_local std::string g_err;

#define BP_EXIT_ON(call)                                                                      \
    do {                                                                                      \
        hipError_t e_ = (call);                                                               \
        if (e_ != hipSuccess) {                                                               \
            fprintf(stderr, "HIP error at %s:%d - %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(EXIT_FAILURE);                                                               \
        }                                                                                     \
    } while (0)

#define BP_RET_ON(call)                                                                       \
    do {                                                                                      \
        hipError_t e_ = (call);                                                               \
        if (e_ != hipSuccess) {                                                               \
            g_err = std::string(#call) + ": " + hipGetErrorString(e_);                       \
            return HIPBP_ERR_DEVICE;                                                          \
        }                                                                                     \
    } while (0)

struct Buf {
    void* p = nullptr;
    size_t cap = 0;
    hipError_t need(size_t bytes) {
        if (bytes <= cap) return hipSuccess;
        if (p) {
            hipError_t e = hipFree(p);
            if (e != hipSuccess) return e;
            p = nullptr;
            cap = 0;
        }
        hipError_t e = hipMalloc(&p, bytes);
        if (e == hipSuccess) cap = bytes;
        return e;
    }
    template <class T>
    T* as() const { return (T*)p; }
};

// HIP-event timing of the verify pipeline's kernels (bench.py's live roofline numbers).
struct EventTimer {
    struct Rec {
        int kind;
        hipEvent_t a, b;
    };
    bool on = false;
    std::vector<hipEvent_t> pool;
    size_t used = 0;
    std::vector<Rec> pending;
    hipEvent_t open[bp::KT_COUNT] = {};
    double total_ms[bp::KT_COUNT] = {};
    uint64_t count[bp::KT_COUNT] = {};

    hipEvent_t get() {
        if (used == pool.size()) {
            hipEvent_t e;
            if (hipEventCreate(&e) != hipSuccess) return nullptr;
            pool.push_back(e);
        }
        return pool[used++];
    }
    void mark(int kind, bool end, hipStream_t s) {
        hipEvent_t e = get();
        if (!e) return;
        (void)hipEventRecord(e, s);
        if (!end)
            open[kind] = e;
        else
            pending.push_back(Rec{kind, open[kind], e});
    }
    hipError_t collect() {
        for (auto& r : pending) {
            hipError_t err = hipEventSynchronize(r.b);
            if (err != hipSuccess) return err;
            float ms = 0;
            if ((err = hipEventElapsedTime(&ms, r.a, r.b)) != hipSuccess) return err;
            total_ms[r.kind] += ms;
            count[r.kind]++;
        }
        pending.clear();
        used = 0;
        return hipSuccess;
    }
    void reset() {
        pending.clear();
        used = 0;
        for (int i = 0; i < bp::KT_COUNT; i++) { total_ms[i] = 0; count[i] = 0; }
    }
};

// Per-device state. The identity-doubling and power-of-two tables are built on first use and cached.
struct Engine {
    EventTimer timer;
    int device = -1;
    hipStream_t stream = nullptr;
    bp::ge* dtab = nullptr;
    bp::fe* two_i = nullptr;
    int two_cap = 0;
    // single-call staging (Part 1: the engine's own stream, synchronous calls)
    Buf h2d[8], scratch[8];
    // hipbp_batch_range_proof_verify_host: a second stream (chunks alternate over two pipelines)
    // and grow-only staging (pinned host + device), reused across calls
    hipStream_t stream2 = nullptr;
    Buf host_dev;
    uint8_t* host_pinned = nullptr;
    size_t host_pinned_cap = 0;
    // ... and the fixed-base prefix tables of the last generator set it saw (G | H | h, h standing
    // in for g, which cuda_range_proof_verify does not read), kept across calls: a caller verifying
    // batch after batch against one generator set builds them once.  Keyed by the generators' bytes
    // (an exact compare of the host copy).  HIPBP_HOST_PREFIX_BITS: 16 by default (1.1 GB at n = 64,
    // built in ~10 ms; fewer bits for larger n, at most 1.25 GB), 0 turns the tables off.
    std::vector<uint8_t> host_gens_key;
    Buf host_gens, host_tab;
    int host_tab_bits = 0;
    // MSM / point-tree workspaces, one set per stream: the Part-2 calls run asynchronously on
    // the caller's stream, so two MSMs on two streams (or an async MSM and a Part-1 call on the
    // engine stream) must never share buffers.  [0] per-point terms, [1..2] block roots,
    // [3..4] tree ping-pong, [5] lane order, [6] sort bins.
    struct MsmBufs { Buf b[7]; };
    std::map<hipStream_t, MsmBufs*> msm_ws;
    Buf* msm_bufs(hipStream_t s) {
        MsmBufs*& m = msm_ws[s];
        if (!m) m = new MsmBufs();
        return m->b;
    }
    // prover workspaces (hipbp_batch_generate_range_proof), one per stream so batches on
    // different streams overlap (one batch's latency-bound stages under another's term launch)
    struct ProverBufs {
        Buf b[19];
    };
    std::map<hipStream_t, ProverBufs*> provers;
    // the generators (G | H | h) a single-proof call last uploaded to h2d[4], as host bytes: the next
    // call with the same bytes (the reference's caller passes one generator set call after call)
    // skips their three pageable copies
    std::vector<uint8_t> single_gens;
    const void* single_gens_dev = nullptr;
    // pinned host staging for the single-proof entry points (a pageable source of an
    // async copy must outlive the copy; this one does, and the stream is synced after use)
    uint8_t* pinned = nullptr;
    size_t pinned_cap = 0;
    hipError_t need_pinned(size_t bytes) {
        if (bytes <= pinned_cap) return hipSuccess;
        hipError_t r;
        if (pinned && (r = hipStreamSynchronize(stream)) != hipSuccess) return r;
        if (pinned && (r = hipHostFree(pinned)) != hipSuccess) return r;
        pinned = nullptr;
        pinned_cap = 0;
        if ((r = hipHostMalloc(&pinned, bytes)) != hipSuccess) return r;
        pinned_cap = bytes;
        return hipSuccess;
    }
    // one-shot verify pipelines, per (stream, n, mode), so batches on different streams overlap
    std::map<std::tuple<hipStream_t, int, int>, struct Pipeline*> pipes;
    std::mutex mu;

    hipError_t init() {
        int dev = 0;
        hipError_t e = hipGetDevice(&dev);
        if (e != hipSuccess) return e;
        device = dev;
        if ((e = hipStreamCreateWithFlags(&stream, hipStreamNonBlocking)) != hipSuccess) return e;
        if ((e = hipMalloc(&dtab, 258 * sizeof(bp::ge))) != hipSuccess) return e;
        // dtab[k] = the identity doubled k times (ge25519_scalarmult's leading zeros), [257] = the
        // host-normalized [256]: computed here with the C forms of the same arithmetic (the device asm
        // forms equal them bit for bit, tests/test_generated_asm.py, asm_check), so a one-proof call
        // launches no set-up kernel and loads no code object besides its own ticks'
        std::vector<bp::ge> t(258);
        t[0] = bp::ge_zero();
        for (int k = 1; k <= 256; k++) t[k] = bp::ge_add(t[k - 1], t[k - 1]);
        t[257] = bp::ge_norm_host(t[256]);
        if ((e = upload(dtab, t.data(), t.size() * sizeof(bp::ge))) != hipSuccess) return e;
        return ensure_two(64);   // grows with the largest n a call brings
    }
    // Host -> device (bytes a multiple of 16), synchronously: staged in the pinned buffer and read from
    // there by a kernel (launch_upload), not by a copy-engine transfer (the process's first
    // hipMemcpyAsync of these 33 KB cost ~7 ms on the first call's path).  The stream is drained
    // first: a caller's own staged copy out of `pinned` may still be queued on it.
    hipError_t upload(void* dst, const void* src, size_t bytes) {
        if (bytes % 16) return hipErrorInvalidValue;   // (whole uint4s: the tables are 32- / 128-B records)
        hipError_t e;
        if ((e = hipStreamSynchronize(stream)) != hipSuccess) return e;
        if ((e = need_pinned(bytes)) != hipSuccess) return e;
        memcpy(pinned, src, bytes);
        bp::launch_upload(dst, pinned, bytes, stream);
        if ((e = hipGetLastError()) != hipSuccess) return e;
        return hipStreamSynchronize(stream);
    }
    // two_i[i] = i successive fe_mul(., 2) from 1 (bulletproof_range_proof.cu:705-712): a grow-only
    // table, extended on the host (C forms) and uploaded whole on growth.  The old device buffer is
    // retired, never freed: ticks and prover launches already queued on OTHER streams (user
    // pipelines, caller prover streams) may still read it, and upload() drains only the engine
    // stream.  Growth doubles, so the retired buffers total less than the live one (a few KB).
    std::vector<bp::fe> two_host;
    std::vector<bp::fe*> two_retired;
    hipError_t ensure_two(int n) {
        if (n <= two_cap) return hipSuccess;
        hipError_t e;
        const int cap = std::max(n, 2 * two_cap);
        const bp::fe two = bp::fe_add(bp::fe_set(1), bp::fe_set(1));
        while ((int)two_host.size() < cap)
            two_host.push_back(two_host.empty() ? bp::fe_set(1) : bp::fe_mul(two_host.back(), two));
        bp::fe* nt = nullptr;
        if ((e = hipMalloc(&nt, (size_t)cap * sizeof(bp::fe))) != hipSuccess) return e;
        if ((e = upload(nt, two_host.data(), (size_t)cap * sizeof(bp::fe))) != hipSuccess) return e;
        if (two_i) two_retired.push_back(two_i);
        two_i = nt;
        two_cap = cap;
        return hipSuccess;
    }
};

Engine* engines[64] = {};
std::mutex engines_mu;

Engine* engine_or_null(hipError_t* err) {
    int dev = 0;
    *err = hipGetDevice(&dev);
    if (*err != hipSuccess) return nullptr;
    if (dev < 0 || dev >= 64) {
        *err = hipErrorInvalidDevice;
        return nullptr;
    }
    std::lock_guard<std::mutex> lk(engines_mu);
    if (!engines[dev]) {
        Engine* e = new Engine();
        *err = e->init();
        if (*err != hipSuccess) {
            delete e;
            return nullptr;
        }
        engines[dev] = e;
    }
    return engines[dev];
}

Engine& engine_or_exit() {
    hipError_t err;
    Engine* e = engine_or_null(&err);
    BP_EXIT_ON(err);
    return *e;
}

// Part-2 entry points run on the caller's stream; NULL is the default (null) stream, as for a
// kernel launch — the stream torch reports as 0 — so work stays ordered with the caller's.
inline hipStream_t pick(void* s, Engine&) { return (hipStream_t)s; }

bool is_pow2(size_t n) { return n && !(n & (n - 1)); }

constexpr size_t MAX_N = size_t(1) << 16;   // generators per proof (range bits / IPA length)

int log2i(size_t n) {
    int k = 0;
    while ((size_t(1) << k) < n) k++;
    return k;
}

int check_batch(const hipbp_proof_batch* b, int range_mode) {
    if (!b) { g_err = "null batch"; return HIPBP_ERR_ARG; }
    if (b->count == 0) return HIPBP_OK;
    if (!is_pow2(b->n) || b->n > MAX_N) { g_err = "n must be a power of two <= 65536"; return HIPBP_ERR_ARG; }
    if (b->ab_len < 1) { g_err = "ab_len must be >= 1"; return HIPBP_ERR_ARG; }
    if ((int)b->L_len > log2i(b->n)) { g_err = "L_len > log2(n)"; return HIPBP_ERR_ARG; }
    if (b->count > (size_t)1 << 24) { g_err = "batch too large"; return HIPBP_ERR_ARG; }
    if (!b->a || !b->b || !b->c || !b->x || (b->L_len && (!b->L || !b->R))) { g_err = "null ipa field"; return HIPBP_ERR_ARG; }
    if (range_mode && (!b->V || !b->A || !b->S || !b->T1 || !b->T2 || !b->t)) { g_err = "null range field"; return HIPBP_ERR_ARG; }
    if (range_mode == 2 && (!b->taux || !b->mu)) { g_err = "range_proof_verify semantics need taux and mu"; return HIPBP_ERR_ARG; }
    return HIPBP_OK;
}

bp::BatchView view_of(const hipbp_proof_batch* b) {
    bp::BatchView v;
    v.B = (int)b->count;
    v.n = (int)b->n;
    v.ab_len = (int)b->ab_len;
    v.L_len = (int)b->L_len;
    v.V = (const bp::ge*)b->V; v.A = (const bp::ge*)b->A; v.S = (const bp::ge*)b->S;
    v.T1 = (const bp::ge*)b->T1; v.T2 = (const bp::ge*)b->T2;
    v.t = (const bp::fe*)b->t; v.a = (const bp::fe*)b->a; v.b = (const bp::fe*)b->b;
    v.c = (const bp::fe*)b->c; v.x = (const bp::fe*)b->x;
    v.L = (const bp::ge*)b->L; v.R = (const bp::ge*)b->R;
    v.taux = (const bp::fe*)b->taux; v.mu = (const bp::fe*)b->mu; v.Vp = (const bp::ge*)b->Vp;
    return v;
}

// The verify pipeline: a ring of D batch slots.  Every tick is ONE k_terms launch over all
// in-flight batches, each at its own stage; within a batch the reference's order is kept
// exactly, across batches nothing depends on anything.  Stages of a batch with L fold rounds
// (Pipeline::stages):
//   0: RK_PREP (challenges, MSM scalars, round challenges)
//   1: RK_STAGE0 (both MSMs' point terms, fold round 0, t*h, c*Q [, the 7 polynomial terms])
//   2: RK_TREE (MSM trees of n > LANE_TREE_MAX points) [, RK_POLY]   r+1 (1 <= r < L): RK_ROUND r
//   FT = L+1 (1 when L = 0): RK_FINAL_TERMS           mode 2, max(3, FT): RK_M3
//   min(3, FIN - 1): RK_LTREE (the trees of n <= LANE_TREE_MAX MSMs, one lane per proof)
//   FIN = 1 + the last of those: RK_FINAL (P, check point, accept)
// Ticks too small to fill the SIMDs (a drain's last ticks, a one-proof verify) run in the lane-quad
// form (QUAD_MAX_ITEMS below).
// A round-r item forms its own input point G'/H' from two round r-1 terms (each folded point
// has exactly one consumer), so no launch of its own is needed for the fold combinations.
// A generator set (hipbp_gens_create): a device snapshot of G[n] | H[n] | h | g and, optionally,
// their fixed-base prefix tables (bp::launch_prefix_tables, same base order).
struct Gens {
    int device = -1;
    size_t n = 0;
    Buf gen, tab;
    int bits = 0;
    const bp::ge* G() const { return gen.as<bp::ge>(); }
    const bp::ge* H() const { return gen.as<bp::ge>() + n; }
    const bp::ge* h() const { return gen.as<bp::ge>() + 2 * n; }
    const bp::ge* g() const { return gen.as<bp::ge>() + 2 * n + 1; }
    void release() {
        if (gen.p) (void)hipFree(gen.p);
        if (tab.p) (void)hipFree(tab.p);
        gen.p = tab.p = nullptr;
    }
};

// Drain-tick thresholds (Pipeline::push): ticks with at most this many scalar-multiplication items
// run them on lane quads, up to PAIR_MAX_ITEMS on lane pairs.  The cost model (tools/ubench_issue.hip
// with -DLAT: one wave alone issues one instruction per ~9 cycles, the SIMD one per ~4.4): a tick
// lasts about (instructions per wave) x max(9, 4.4 w) cycles for w waves per SIMD, counting the other
// pipeline's concurrent tick (they drain side by side).  Quads cut the instructions per wave of a
// point operation from ~1700 to ~750 for 4x the lanes, pairs to ~1140 for 2x: with both pipelines'
// drains together, a 65,536-item tick is fastest on lanes, 32,768 on pairs, 16,384 on quads
// (configs[4] shard: 173.8 K verifies/s vs 172.1 K with the round-3 bounds 49,152 / 98,304).
// 16-lane rows (sm_row) up to this many items: a one-proof call's ticks (r04b, one MI355X, warm
// cuda_range_proof_verify: n = 16 4.9 -> 4.0 ms, n = 64 6.7 -> 5.5 ms)
constexpr unsigned long long ROW_MAX_ITEMS = 2048;
constexpr unsigned long long QUAD_MAX_ITEMS = 16384;
constexpr unsigned long long PAIR_MAX_ITEMS = 32768;

struct Pipeline {
    Engine* e = nullptr;
    hipStream_t s = nullptr;
    int n = 0, Lr = 0, D = 0;
    size_t maxB = 0;
    int range_mode = 1;   // 0 inner product only, 1 cuda_range_proof_verify, 2 range_proof_verify
    const bp::ge *G = nullptr, *H = nullptr, *g = nullptr, *h = nullptr;
    struct Slot {
        Buf b[24];
        bp::SlotDev dev{};
        bool active = false;
        int stage = 0;
        size_t B = 0;
        hipEvent_t copied = nullptr;
    };
    std::vector<Slot> slots;
    bp::SlotDev* slots_dev = nullptr;   // device copies [D]
    bp::SlotDev* host_dev = nullptr;    // pinned staging [D]
    int head = 0;

    struct Stages {
        int ft, m3, fin;
    };
    Stages stages(int L) const {
        Stages g;
        g.ft = L > 0 ? L + 1 : 1;
        g.m3 = range_mode == 2 ? (g.ft > 3 ? g.ft : 3) : -1;
        int last = g.ft;
        if (range_mode && last < 2) last = 2;       // the MSM trees (RK_TREE blocks when n > LANE_TREE_MAX)
        if (g.m3 > last) last = g.m3;
        g.fin = last + 1;
        return g;
    }
    // Layout switches (A/B runs in round 1; defaults = the measured best on MI355X,
    // 138.7K verifies/s lane trees + chains last vs 137.9K block trees, 130.6K lane trees + chains
    // first): HIPBP_LANE_TREE_MAX (lane trees for n <= it), HIPBP_CHAINS_FIRST (per-proof chain
    // regions at the start of the grid instead of the end).
    bool lane_tree = false, chains_first = false;
    // Split stage 0 ("deferred MSM terms", hipbp_pipeline_defer_msm / HIPBP_DEFER_MSM=1): a batch
    // pushed with it on runs only fold round 0 (+ the polynomial terms) in its stage-0 tick; its
    // MSM terms, t*h and c*Q (read only by the lane trees and the final assembly) run as RK_MSMT
    // chunks inside its fold-round ticks (stages 2 .. L), whose items shrink round by round, and
    // the lane trees move to the stage after the last chunk (the final-terms tick).  For a finite batch
    // (configs[4]'s shards) the rounds that would run half empty before the latency-bound last
    // ticks carry the MSM work instead.  Needs the lane trees (n <= 64) and L >= 2.
    bool defer_msm = false;
    // drain-tick forms (push): HIPBP_QUAD forces lanes (0) / quads (1) / pairs (2) on every tick
    // (-1: by size), HIPBP_QUAD_MAX_ITEMS / HIPBP_PAIR_MAX_ITEMS move the size bounds
    int quad_force = -1;
    unsigned long long row_max = ROW_MAX_ITEMS, quad_max = QUAD_MAX_ITEMS, pair_max = PAIR_MAX_ITEMS;
    // Lane sort (bp::launch_lane_sort): per-lane-scalar items in chain-length order, for batches
    // of at least LANE_SORT_MIN proofs (HIPBP_LANE_SORT=0 turns it off, for A/B runs).
    static constexpr size_t LANE_SORT_MIN = 64;
    bool lane_sort = true;
    int lane_sort_mask = 7;   // bit 0 stage 0, bit 1 rounds, bit 2 final terms, bit 3 shortest first
    Buf sort_bins, sort_offs;
    bp::LaneSortPlan plan{};
    // HIPBP_SORT_STREAM=1: the lane sort's three small launches on a high-priority stream of their
    // own (between two events), so a concurrent pipeline's big tick cannot starve them of workgroup
    // slots (a 4096-proof shard batch's sort once waited 7 ms behind the other pipeline's stage 0).
    // Off by default since the sort runs in 256-thread blocks, which fit beside a running tick:
    // then 172.5 vs 171.5 K (shard) and 190.4 vs 189.5 K (headline) verifies/s without it.
    hipStream_t sort_s = nullptr;
    hipEvent_t ev_tick = nullptr, ev_sorted = nullptr;
    // fixed-base prefix tables of G, H, h, g (hipbp_pipeline_prefix_tables: ptab, owned; or a
    // generator set's, hipbp_pipeline_use_gens: ext_tab, borrowed); pbits = 0: none
    Buf ptab;
    const bp::ge* ext_tab = nullptr;
    int pbits = 0;
    const bp::ge* tables() const { return ext_tab ? ext_tab : ptab.as<bp::ge>(); }
    hipError_t init(Engine* eng, hipStream_t st, size_t mb, int nn, int range) {
        e = eng; s = st; maxB = mb; n = nn; range_mode = range;
        const char* ls = getenv("HIPBP_LANE_SORT");
        lane_sort_mask = ls ? atoi(ls) : 7;
        lane_sort = (lane_sort_mask & 7) != 0;
        const char* lt = getenv("HIPBP_LANE_TREE_MAX");
        lane_tree = n <= (lt ? atoi(lt) : bp::LANE_TREE_MAX);
        const char* cf = getenv("HIPBP_CHAINS_FIRST");
        chains_first = cf ? atoi(cf) != 0 : false;
        // drain-tick form knobs, read once per pipeline (push runs on the issue path)
        const char* qe = getenv("HIPBP_QUAD");
        const char* qm = getenv("HIPBP_QUAD_MAX_ITEMS");
        const char* pm = getenv("HIPBP_PAIR_MAX_ITEMS");
        quad_force = qe ? (atoi(qe) == 1 ? 4 : atoi(qe) == 2 ? 2 : atoi(qe) == 3 ? 16 : 1) : -1;
        const char* rm = getenv("HIPBP_ROW_MAX_ITEMS");
        row_max = rm ? strtoull(rm, nullptr, 10) : ROW_MAX_ITEMS;
        quad_max = qm ? strtoull(qm, nullptr, 10) : QUAD_MAX_ITEMS;
        pair_max = pm ? strtoull(pm, nullptr, 10) : PAIR_MAX_ITEMS;
        const char* dm = getenv("HIPBP_DEFER_MSM");
        defer_msm = dm && atoi(dm) != 0;
        if (const char* sp = getenv("HIPBP_DEFER_SPAN")) {
            int a = 2, b = 1, c = 0;
            if (sscanf(sp, "%d:%d:%d", &a, &b, &c) >= 1 && a >= 2) {
                defer_first = a;
                defer_last_off = b < 0 ? 0 : b;
                defer_weight = c != 0;
            }
        }
        Lr = log2i((size_t)n);
        D = stages(Lr).fin + 1;   // batches with fewer rounds finish earlier
        slots.resize(D);
        hipError_t r;
        if ((r = hipMalloc(&slots_dev, D * sizeof(bp::SlotDev))) != hipSuccess) return r;
        if ((r = hipHostMalloc(&host_dev, D * sizeof(bp::SlotDev))) != hipSuccess) return r;
        for (auto& sl : slots)
            if ((r = hipEventCreateWithFlags(&sl.copied, hipEventDisableTiming)) != hipSuccess) return r;
        const char* ss = getenv("HIPBP_SORT_STREAM");
        if (ss && atoi(ss) != 0) {
            int lo_pr = 0, hi_pr = 0;
            if ((r = hipDeviceGetStreamPriorityRange(&lo_pr, &hi_pr)) != hipSuccess) return r;
            if ((r = hipStreamCreateWithPriority(&sort_s, hipStreamNonBlocking, hi_pr)) != hipSuccess) return r;
            if ((r = hipEventCreateWithFlags(&ev_tick, hipEventDisableTiming)) != hipSuccess) return r;
            if ((r = hipEventCreateWithFlags(&ev_sorted, hipEventDisableTiming)) != hipSuccess) return r;
        }
        return hipSuccess;
    }
    void release() {
        if (s) (void)hipStreamSynchronize(s);
        for (auto& sl : slots) {
            for (auto& b : sl.b) if (b.p) (void)hipFree(b.p);
            if (sl.copied) (void)hipEventDestroy(sl.copied);
        }
        if (slots_dev) (void)hipFree(slots_dev);
        if (host_dev) (void)hipHostFree(host_dev);
        if (sort_s) (void)hipStreamSynchronize(sort_s);
        if (sort_s) (void)hipStreamDestroy(sort_s);
        if (ev_tick) (void)hipEventDestroy(ev_tick);
        if (ev_sorted) (void)hipEventDestroy(ev_sorted);
        if (sort_bins.p) (void)hipFree(sort_bins.p);
        if (sort_offs.p) (void)hipFree(sort_offs.p);
        if (ptab.p) (void)hipFree(ptab.p);
    }
    // The batch's per-lane item sets (stage 0's per-lane part, the rounds whose scalar runs are
    // shorter than a wave, the final terms), their lane-order buffers and the sort plan.
    hipError_t plan_sort(Slot& sl, int idx) {
        plan = bp::LaneSortPlan{};
        bp::SlotDev& d = sl.dev;
        d.perm0 = nullptr;
        for (auto& q : d.permr) q = nullptr;
        d.perm_ft = nullptr;
        const unsigned long long B = d.bv.B;
        const int L = d.bv.L_len;
        if (!lane_sort || B < LANE_SORT_MIN) return hipSuccess;
        struct S { int kind, r; unsigned long long items; };
        S sets[bp::LANE_SORT_SETS];
        int cnt = 0;
        const bp::Stage0Lanes z = bp::stage0_lanes(B, n, L, range_mode);
        for (int c = 0; c < 4; c++)   // one set per class, contiguous in perm0 (stage0_item)
            if (z.size[c] && (lane_sort_mask & 1)) sets[cnt++] = {bp::SS_STAGE0, c, z.size[c]};
        for (int r = 1; r < L; r++)
            if (bp::round_per_lane(n, r) && (lane_sort_mask & 2))
                sets[cnt++] = {bp::SS_ROUND, r, B * 4 * (unsigned long long)(n >> (r + 1))};
        if (lane_sort_mask & 4) sets[cnt++] = {bp::SS_FT, 0, B * 2};
        if (!cnt) return hipSuccess;
        plan.longest_first = (lane_sort_mask & 8) ? 0 : 1;
        unsigned long long total = 0;
        for (int k = 0; k < cnt; k++) total += sets[k].items;
        if (total > 0xFFFFFFFFull) return hipSuccess;
        hipError_t r;
        if ((r = sl.b[20].need(total * sizeof(uint32_t))) != hipSuccess) return r;
        const size_t nb = (size_t)bp::LANE_SORT_SETS * bp::MSM_BINS * sizeof(unsigned);
        if (!sort_bins.p) {
            if ((r = sort_bins.need(nb)) != hipSuccess) return r;
            if ((r = hipMemsetAsync(sort_bins.p, 0, nb, s)) != hipSuccess) return r;
            if ((r = sort_offs.need(nb)) != hipSuccess) return r;
        }
        uint32_t* base = sl.b[20].as<uint32_t>();
        unsigned blk = 0;
        for (int k = 0; k < cnt; k++) {
            bp::LaneSortPlan::Set& st = plan.set[k];
            st.kind = sets[k].kind; st.r = sets[k].r; st.items = sets[k].items; st.perm = base; st.block0 = blk;
            if (st.kind == bp::SS_STAGE0 && !d.perm0) d.perm0 = base;
            else if (st.kind == bp::SS_ROUND) d.permr[st.r] = base;
            else d.perm_ft = base;
            base += sets[k].items;
            blk += (unsigned)((sets[k].items + bp::LANE_SORT_BLOCK - 1) / bp::LANE_SORT_BLOCK);
        }
        plan.count = cnt;
        plan.blocks = blk;
        plan.slot = slots_dev + idx;
        return hipSuccess;
    }
    bool busy() const {
        for (auto& sl : slots) if (sl.active) return true;
        return false;
    }
    // A split batch adds one RK_MSMT region to each of its stages 2 .. L: in steady state a tick then
    // holds up to 2 L + 5 regions (RK_STAGE0, L - 1 RK_ROUND + L - 1 RK_MSMT, RK_FINAL_TERMS, RK_M3,
    // RK_FINAL, RK_LTREE, RK_POLY, RK_PREP), which must fit the kernel's region list (n <= 512 when
    // HIPBP_LANE_TREE_MAX raises the lane-tree limit; the default limit is n <= 64, 17 regions).
    bool defer_ok() const { return range_mode != 0 && lane_tree && Lr >= 2 && 2 * Lr + 5 <= bp::MAX_REGIONS; }
    // a split batch's MSM-term chunks: stages defer_first .. msm_last(L), wave-aligned lane ranges
    // (HIPBP_DEFER_SPAN = "first:last_off:weight" for A/B runs: chunks at stages first .. L - last_off
    // (at least first), weight 0 equal chunks, 1 chunk k weighted 2^k: later, emptier rounds get more)
    // default 2:0:0 (r04k, 8192-proof shard: 180.7 / 181.2 K vs 178.4 / 178.2 K with 2:1:0)
    int defer_first = 2, defer_last_off = 0, defer_weight = 0;
    int msm_last(int L) const { return L - defer_last_off > defer_first ? L - defer_last_off : defer_first; }
    void msm_chunk(unsigned long long total, int L, int st, unsigned long long& lo, unsigned long long& hi) const {
        const int m = msm_last(L) - defer_first + 1, k = st - defer_first;   // m chunks, this is chunk k
        auto cut = [&](int j) -> unsigned long long {   // lanes before chunk j
            if (j >= m) return total;
            const unsigned long long num = defer_weight ? (1ull << j) - 1 : (unsigned long long)j;
            const unsigned long long den = defer_weight ? (1ull << m) - 1 : (unsigned long long)m;
            return (total / 64 * num / den) * 64;
        };
        lo = cut(k);
        hi = cut(k + 1);
    }
    int ltree_stage(const Slot& sl, const Stages& g) const {
        return sl.dev.defer ? msm_last(sl.dev.bv.L_len) + 1 : std::min(3, g.fin - 1);
    }
    hipError_t carve(Slot& sl, size_t B, size_t Lb) {
        hipError_t r;
        size_t Lc = Lb ? Lb : 1;
        size_t sz[14] = {B * 32, B * n * 32, B * 4 * 32, B * Lc * 32, B * Lc * 32, B, B * 2 * n * 128, B * 2 * 128,
                         B * 4 * 128, B * 2 * n * 128, B * 2 * n * 128, 0, B * 2 * 128, B * 128};
        for (int i = 0; i < 14; i++)
            if ((r = sl.b[i].need(sz[i])) != hipSuccess) return r;
        bp::VerifyWs& w = sl.dev.ws;
        w.sG = sl.b[0].as<bp::fe>(); w.sH = sl.b[1].as<bp::fe>(); w.sc = sl.b[2].as<bp::fe>();
        w.u = sl.b[3].as<bp::fe>(); w.uinv = sl.b[4].as<bp::fe>(); w.ipok = sl.b[5].as<uint8_t>();
        w.msm_pts = sl.b[6].as<bp::ge>(); w.msm_part = sl.b[7].as<bp::ge>(); w.terms = sl.b[8].as<bp::ge>();
        w.fold[0] = sl.b[9].as<bp::ge>(); w.fold[1] = sl.b[10].as<bp::ge>();
        w.fin = sl.b[12].as<bp::ge>(); w.Pin = sl.b[13].as<bp::ge>();
        if (range_mode == 2) {
            size_t sz2[6] = {B * 8 * 32, B * 8 * 128, B * 2 * 128, B * 32, B * 2 * 128, B};
            for (int i = 0; i < 6; i++)
                if ((r = sl.b[14 + i].need(sz2[i])) != hipSuccess) return r;
            if ((r = sl.b[21].need(B * 3 * 128)) != hipSuccess) return r;
            w.psc = sl.b[14].as<bp::fe>(); w.pterm = sl.b[15].as<bp::ge>(); w.lr = sl.b[16].as<bp::ge>();
            w.chal = sl.b[17].as<bp::fe>(); w.m3 = sl.b[18].as<bp::ge>(); w.rflags = sl.b[19].as<uint8_t>();
            w.pbase = sl.b[21].as<bp::ge>();
        } else {
            w.psc = nullptr; w.pterm = nullptr; w.lr = nullptr; w.chal = nullptr; w.m3 = nullptr; w.rflags = nullptr;
            w.pbase = nullptr;
        }
        return hipSuccess;
    }

    // One tick; `b` may be null (drain).  Outputs of `b` are written when it completes.
    int push(const hipbp_proof_batch* b, const ge25519* P_in, uint8_t* ok, ge25519* P_out, ge25519* chk,
             uint8_t* flags_out = nullptr, ge25519* poly_out = nullptr) {
        EventTimer* tm = e->timer.on ? &e->timer : nullptr;
        bool has = b && b->count > 0;
        Slot& nw = slots[head];
        if (has) {
            int rc = check_batch(b, range_mode);
            if (rc != HIPBP_OK) return rc;
            if ((int)b->n != n) { g_err = "batch n differs from the pipeline's"; return HIPBP_ERR_ARG; }
            if (nw.active) { g_err = "pipeline slot busy (internal)"; return HIPBP_ERR_ARG; }
            BP_RET_ON(carve(nw, b->count, b->L_len));
            nw.dev.bv = view_of(b);
            nw.dev.ok = ok;
            nw.dev.P_out = (bp::ge*)P_out;
            nw.dev.chk_out = (bp::ge*)chk;
            nw.dev.flags_out = flags_out;
            nw.dev.poly_out = (bp::ge*)poly_out;
            nw.dev.range_mode = range_mode;
            nw.dev.lane_tree = lane_tree ? 1 : 0;
            nw.dev.ptab = pbits ? tables() : nullptr;
            nw.dev.pbits = pbits;
            // (the lane trees must land at least one tick before the final assembly)
            nw.dev.defer = (defer_msm && defer_ok() && (int)b->L_len >= 2 &&
                            msm_last((int)b->L_len) + 1 < stages((int)b->L_len).fin) ? 1 : 0;
            BP_RET_ON(plan_sort(nw, head));
            BP_RET_ON(hipEventSynchronize(nw.copied));   // staging slot free again
            host_dev[head] = nw.dev;
            BP_RET_ON(hipMemcpyAsync(slots_dev + head, host_dev + head, sizeof(bp::SlotDev), hipMemcpyHostToDevice, s));
            BP_RET_ON(hipEventRecord(nw.copied, s));
            if (!range_mode)
                BP_RET_ON(hipMemcpyAsync(nw.dev.ws.Pin, P_in, b->count * sizeof(ge25519), hipMemcpyDeviceToDevice, s));
            nw.active = true;
            nw.stage = 0;
            nw.B = b->count;
        }
        bp::RegionList tr{};
        bool overflow = false;
        auto add = [&overflow](bp::RegionList& rl, int kind, int slot, int r, unsigned long long items, unsigned align) {
            if (!items) return;
            if (rl.count == bp::MAX_REGIONS) { overflow = true; return; }
            bp::Region& g = rl.reg[rl.count++];
            g.kind = kind; g.slot = slot; g.r = r; g.begin = rl.total; g.items = items;
            rl.total += (items + align - 1) & ~(unsigned long long)(align - 1);   // wave / block aligned
        };
        // pass 0: the (block-aligned) tree region, which must start the list; pass 2: the scalar
        // multiplications; the per-proof chains (final assembly incl. lane trees, polynomial
        // sides, challenges) in pass 3 by default (measured faster than pass 1, the grid start)
        const int chain_pass = chains_first ? 1 : 3;
        for (int pass = 0; pass < 4; pass++) {
            for (int k = 0; k < D; k++) {
                int idx = (head - k + D) % D;   // newest first
                Slot& sl = slots[idx];
                if (!sl.active) continue;
                unsigned long long B = sl.dev.bv.B;
                int L = sl.dev.bv.L_len, st = sl.stage;
                const Stages g = stages(L);
                if (pass == 0) {
                    if (st == 2 && range_mode && !lane_tree) add(tr, bp::RK_TREE, idx, 0, B * 2 * n, 256);
                } else if (pass == chain_pass) {
                    if (st == g.fin) add(tr, bp::RK_FINAL, idx, 0, B, 64);
                    // the lane MSM trees need only stage 0's terms: a few ticks before the final one,
                    // so a drain's last tick is the short P / check-point assembly alone
                    if (range_mode && lane_tree && st == ltree_stage(sl, g)) {
                        add(tr, bp::RK_LTREE, idx, 0, B, 64);
                    }
                    if (st == 2 && range_mode == 2) add(tr, bp::RK_POLY, idx, 0, B, 64);
                    if (st == 0) add(tr, bp::RK_PREP, idx, 0, range_mode ? 2 * B : B, 64);
                } else if (pass == 2) {
                    if (st == 1) {
                        add(tr, bp::RK_STAGE0, idx, 0,
                            bp::stage0_lanes(B, n, L, range_mode, sl.dev.defer ? bp::S0_CRIT : bp::S0_ALL).total, 64);
                    }
                    if (st >= 2 && st <= L) add(tr, bp::RK_ROUND, idx, st - 1, B * 4 * (n >> st), 64);
                    if (sl.dev.defer && st >= defer_first && st <= msm_last(L)) {   // a chunk of the split stage 0
                        unsigned long long lo, hi;
                        msm_chunk(bp::stage0_lanes(B, n, L, range_mode, bp::S0_DEFER).total, L, st, lo, hi);
                        add(tr, bp::RK_MSMT, idx, (int)lo, hi - lo, 64);
                    }
                    if (st == g.ft) add(tr, bp::RK_FINAL_TERMS, idx, 0, B * 2, 64);
                    if (st == g.m3) add(tr, bp::RK_M3, idx, 0, B * 2, 64);
                }
            }
        }
        if (overflow) { g_err = "pipeline region list overflow (internal)"; return HIPBP_ERR_ARG; }
        // Drain-tick form: a tick whose scalar multiplications cannot fill the SIMDs (the last
        // fold rounds and final terms of the last batches, a one-proof verify) lasts one
        // scalar-multiplication chain's latency; its items then take a lane quad each (k_terms<4>,
        // 3 product latencies per point op instead of 9).  HIPBP_QUAD=0/1 forces it off/on;
        // HIPBP_QUAD_MAX_ITEMS sets the tick's scalar-multiplication items up to which it is used.
        unsigned long long sm_items = 0;
        for (int k = 0; k < tr.count; k++)
            if (bp::region_is_sm(tr.reg[k].kind)) sm_items += tr.reg[k].items;
        // Between the two (up to PAIR_MAX_ITEMS), lane pairs (HIPBP_QUAD=2 forces them,
        // HIPBP_PAIR_MAX_ITEMS sets the bound).
        int ql = sm_items <= row_max ? 16 : sm_items <= quad_max ? 4 : sm_items <= pair_max ? 2 : 1;
        if (!sm_items) {   // a tick of chains alone: the chains on quads, in the row-form kernel when the
            // tick is small (a one-proof call's ticks then load one tick code object, not two)
            unsigned long long chain_items = 0;
            for (int k = 0; k < tr.count; k++) chain_items += tr.reg[k].items;
            ql = chain_items <= row_max ? 16 : 4;
        }
        if (quad_force >= 0) ql = quad_force;
        if (ql > 1) {   // re-lay the regions: scalar-multiplication items ql lanes each
            unsigned long long tot = 0;
            for (int k = 0; k < tr.count; k++) {
                bp::Region& g = tr.reg[k];
                g.items *= bp::region_lanes(g.kind, ql);
                g.begin = tot;
                const unsigned long long al = g.kind == bp::RK_TREE ? 256 : 64;
                tot += (g.items + al - 1) & ~(al - 1);
            }
            tr.total = tot;
        }
        if (tr.total >= (1ull << 32)) { g_err = "pipeline tick exceeds 2^32 lanes (batch too large for n)"; return HIPBP_ERR_ARG; }
        if (tm) tm->mark(bp::KT_TERMS, false, s);
        bp::launch_terms(tr, slots_dev, G, H, g ? g : h, h, e->dtab, e->two_i, s, ql);
        if (tm) tm->mark(bp::KT_TERMS, true, s);
        BP_RET_ON(hipGetLastError());
        if (has && plan.count) {   // the new batch's scalars exist now (its RK_PREP ran): order its lanes
            if (sort_s) {   // tick -> sort (high priority) -> the pipeline's next tick
                BP_RET_ON(hipEventRecord(ev_tick, s));
                BP_RET_ON(hipStreamWaitEvent(sort_s, ev_tick, 0));
                bp::launch_lane_sort(plan, sort_bins.as<unsigned>(), sort_offs.as<unsigned>(), sort_s);
                BP_RET_ON(hipGetLastError());
                BP_RET_ON(hipEventRecord(ev_sorted, sort_s));
                BP_RET_ON(hipStreamWaitEvent(s, ev_sorted, 0));
            } else {
                bp::launch_lane_sort(plan, sort_bins.as<unsigned>(), sort_offs.as<unsigned>(), s);
                BP_RET_ON(hipGetLastError());
            }
        }
        for (auto& sl : slots) {
            if (!sl.active) continue;
            if (sl.stage == stages(sl.dev.bv.L_len).fin) sl.active = false;
            else sl.stage++;
        }
        head = (head + 1) % D;
        return HIPBP_OK;
    }
    int flush() {
        while (busy()) {
            int rc = push(nullptr, nullptr, nullptr, nullptr, nullptr);
            if (rc != HIPBP_OK) return rc;
        }
        return HIPBP_OK;
    }
};

// `count` canonical-tree MSMs of n points each on stream s, in s's own workspace.
hipError_t msm_run(Engine& e, bp::ge* results, const bp::fe* scalars, const bp::ge* points, size_t n, size_t count,
                   hipStream_t s, const bp::ge* ptab = nullptr, int K = 0) {
    const size_t tot = n * count, nb = count * ((n + 255) / 256);
    Buf* w = e.msm_bufs(s);
    hipError_t err;
    if ((err = w[0].need(tot * sizeof(bp::ge))) != hipSuccess) return err;
    if ((err = w[1].need(nb * sizeof(bp::ge))) != hipSuccess) return err;
    if ((err = w[2].need(nb * sizeof(bp::ge))) != hipSuccess) return err;
    if ((err = w[5].need(tot * sizeof(uint32_t))) != hipSuccess) return err;
    if ((err = w[6].need(bp::MSM_BINS * sizeof(unsigned))) != hipSuccess) return err;
    bp::launch_msm_full(results, scalars, points, n, w[0].as<bp::ge>(), w[1].as<bp::ge>(), w[2].as<bp::ge>(),
                        w[5].as<uint32_t>(), w[6].as<unsigned>(), e.dtab, s, count, ptab, K);
    return hipGetLastError();
}

// The engine's cached one-shot pipeline for (stream, n, mode); created on first use.  Cached only
// once fully initialised (a failed init is released, never reused).
int pipeline_for(Engine& e, hipStream_t s, size_t max_batch, int n, int range_mode, Pipeline** out) {
    auto key = std::make_tuple(s, n, range_mode);
    auto it = e.pipes.find(key);
    if (it != e.pipes.end()) {
        *out = it->second;
        return HIPBP_OK;
    }
    Pipeline* pl = new Pipeline();
    hipError_t ierr = pl->init(&e, s, max_batch, n, range_mode);
    if (ierr != hipSuccess) {
        pl->release();
        delete pl;
        BP_RET_ON(ierr);
    }
    e.pipes[key] = pl;
    *out = pl;
    return HIPBP_OK;
}

// One-shot verify of a whole batch on `s` (push + drain of a cached pipeline).
int run_verify(Engine& e, const hipbp_proof_batch* batch, const ge25519* P_in, const ge25519* G, const ge25519* H,
               const ge25519* h, uint8_t* ok, ge25519* P_out, ge25519* chk_out, int range_mode, hipStream_t s,
               const ge25519* g = nullptr, uint8_t* flags_out = nullptr, ge25519* poly_out = nullptr,
               const bp::ge* tab = nullptr, int tab_bits = 0) {
    int rc = check_batch(batch, range_mode);
    if (rc != HIPBP_OK || batch->count == 0) return rc;
    if (range_mode) BP_RET_ON(e.ensure_two((int)batch->n));
    Pipeline* pl = nullptr;
    if ((rc = pipeline_for(e, s, batch->count, (int)batch->n, range_mode, &pl)) != HIPBP_OK) return rc;
    pl->G = (const bp::ge*)G;
    pl->H = (const bp::ge*)H;
    pl->h = (const bp::ge*)h;
    pl->g = (const bp::ge*)g;
    // a generator set's prefix tables, lent for this call only (the cached pipeline is shared with
    // the calls that have none): the ticks' slot records take the pointer at push
    pl->ext_tab = tab_bits ? tab : nullptr;
    pl->pbits = tab_bits ? tab_bits : 0;
    rc = pl->push(batch, P_in, ok, P_out, chk_out, flags_out, poly_out);
    if (rc == HIPBP_OK) rc = pl->flush();
    pl->ext_tab = nullptr;
    pl->pbits = 0;
    return rc;
}

// ---- host staging for the single-proof reference entry points
struct HostProofStage {
    std::vector<fe25519> a, b;
    std::vector<ge25519> L, R;
};

}  // namespace

extern "C" {

const char* hipbp_last_error(void) { return g_err.c_str(); }

int hipbp_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

int hipbp_sync(void* stream) {
    hipError_t err;
    Engine* e = engine_or_null(&err);
    BP_RET_ON(err);
    BP_RET_ON(hipStreamSynchronize(pick(stream, *e)));
    return HIPBP_OK;
}

static const char* kKernelNames[bp::KT_COUNT] = {"k_prep", "k_terms", "k_tree", "k_combine"};

int hipbp_timing_enable(int on) {
    hipError_t err;
    Engine* e = engine_or_null(&err);
    BP_RET_ON(err);
    std::lock_guard<std::mutex> lk(e->mu);
    BP_RET_ON(e->timer.collect());
    e->timer.reset();
    e->timer.on = on != 0;
    return HIPBP_OK;
}

int hipbp_timing_collect(double* total_ms, uint64_t* launches) {
    hipError_t err;
    Engine* e = engine_or_null(&err);
    BP_RET_ON(err);
    std::lock_guard<std::mutex> lk(e->mu);
    BP_RET_ON(e->timer.collect());
    for (int i = 0; i < bp::KT_COUNT; i++) {
        if (total_ms) total_ms[i] = e->timer.total_ms[i];
        if (launches) launches[i] = e->timer.count[i];
    }
    return HIPBP_OK;
}

int hipbp_kernel_count(void) { return bp::KT_COUNT; }

const char* hipbp_kernel_name(int kind) { return (kind >= 0 && kind < bp::KT_COUNT) ? kKernelNames[kind] : ""; }

int hipbp_batch_range_proof_verify(const hipbp_proof_batch* batch, const ge25519* G, const ge25519* H,
                                   const ge25519* g, const ge25519* h, uint8_t* ok, ge25519* P_out,
                                   ge25519* check_out, void* stream) {
    (void)g;   // g is not read by cuda_range_proof_verify (crv:82-127)
    hipError_t err;
    Engine* e = engine_or_null(&err);
    BP_RET_ON(err);
    if (batch && batch->count == 0) return HIPBP_OK;   // nothing read or written: empty outputs may be null
    if (!G || !H || !h || !ok) { g_err = "null generator/output"; return HIPBP_ERR_ARG; }
    std::lock_guard<std::mutex> lk(e->mu);
    return run_verify(*e, batch, nullptr, G, H, h, ok, P_out, check_out, 1, pick(stream, *e));
}

int hipbp_batch_range_proof_verify_std(const hipbp_proof_batch* batch, const ge25519* G, const ge25519* H,
                                       const ge25519* g, const ge25519* h, uint8_t* ok, ge25519* P_out,
                                       ge25519* check_out, uint8_t* flags_out, ge25519* poly_out, void* stream) {
    hipError_t err;
    Engine* e = engine_or_null(&err);
    BP_RET_ON(err);
    if (batch && batch->count == 0) return HIPBP_OK;   // nothing read or written: empty outputs may be null
    if (!G || !H || !g || !h || !ok) { g_err = "null generator/output"; return HIPBP_ERR_ARG; }
    std::lock_guard<std::mutex> lk(e->mu);
    return run_verify(*e, batch, nullptr, G, H, h, ok, P_out, check_out, 2, pick(stream, *e), g, flags_out,
                      poly_out);
}

int hipbp_batch_range_proof_verify_gens(const hipbp_proof_batch* batch, void* gens, uint8_t* ok, ge25519* P_out,
                                        ge25519* check_out, void* stream) {
    Gens* gs = (Gens*)gens;
    if (!gs) { g_err = "null gens"; return HIPBP_ERR_ARG; }
    hipError_t err;
    Engine* e = engine_or_null(&err);
    BP_RET_ON(err);
    if (batch && batch->count == 0) return HIPBP_OK;   // nothing read or written: empty outputs may be null
    if (!ok) { g_err = "null output"; return HIPBP_ERR_ARG; }
    if (batch && batch->n != gs->n) { g_err = "batch n differs from the generator set's"; return HIPBP_ERR_ARG; }
    if (gs->device != e->device) { g_err = "gens: created on another device"; return HIPBP_ERR_ARG; }
    std::lock_guard<std::mutex> lk(e->mu);
    return run_verify(*e, batch, nullptr, (const ge25519*)gs->G(), (const ge25519*)gs->H(), (const ge25519*)gs->h(),
                      ok, P_out, check_out, 1, pick(stream, *e), nullptr, nullptr, nullptr,
                      gs->bits ? gs->tab.as<bp::ge>() : nullptr, gs->bits);
}

int hipbp_batch_inner_product_verify(const hipbp_proof_batch* batch, const ge25519* P, const ge25519* G,
                                     const ge25519* H, const ge25519* Q, uint8_t* ok, ge25519* check_out,
                                     void* stream) {
    hipError_t err;
    Engine* e = engine_or_null(&err);
    BP_RET_ON(err);
    if (batch && batch->count == 0) return HIPBP_OK;   // nothing read or written: empty outputs may be null
    if (!P || !G || !H || !Q || !ok) { g_err = "null argument"; return HIPBP_ERR_ARG; }
    std::lock_guard<std::mutex> lk(e->mu);
    return run_verify(*e, batch, P, G, H, Q, ok, nullptr, check_out, 0, pick(stream, *e));
}

void* hipbp_pipeline_create(size_t max_batch, size_t n, int range_mode, const ge25519* G, const ge25519* H,
                            const ge25519* g, const ge25519* h, void* stream) {
    hipError_t err;
    Engine* e = engine_or_null(&err);
    if (!e) { g_err = std::string("engine: ") + hipGetErrorString(err); return nullptr; }
    if (!is_pow2(n) || n > MAX_N || !G || !H || !h) { g_err = "pipeline: bad n or null generator"; return nullptr; }
    if (range_mode < 0 || range_mode > 2 || (range_mode == 2 && !g)) { g_err = "pipeline: bad mode or null g"; return nullptr; }
    if (range_mode) {
        std::lock_guard<std::mutex> lk(e->mu);
        if ((err = e->ensure_two((int)n)) != hipSuccess) {
            g_err = std::string("pipeline tables: ") + hipGetErrorString(err);
            return nullptr;
        }
    }
    Pipeline* pl = new Pipeline();
    err = pl->init(e, pick(stream, *e), max_batch, (int)n, range_mode);
    if (err != hipSuccess) {
        g_err = std::string("pipeline init: ") + hipGetErrorString(err);
        pl->release();
        delete pl;
        return nullptr;
    }
    pl->G = (const bp::ge*)G;
    pl->H = (const bp::ge*)H;
    pl->h = (const bp::ge*)h;
    pl->g = (const bp::ge*)g;
    return pl;
}

int hipbp_pipeline_push(void* handle, const hipbp_proof_batch* batch, const ge25519* P_in, uint8_t* ok,
                        ge25519* P_out, ge25519* check_out, uint8_t* flags_out, ge25519* poly_out) {
    Pipeline* pl = (Pipeline*)handle;
    if (!pl) { g_err = "null pipeline"; return HIPBP_ERR_ARG; }
    if (batch && batch->count && (!ok || (!pl->range_mode && !P_in))) { g_err = "null output/P"; return HIPBP_ERR_ARG; }
    std::lock_guard<std::mutex> lk(pl->e->mu);
    return pl->push(batch, P_in, ok, P_out, check_out, flags_out, poly_out);
}

int hipbp_pipeline_flush(void* handle) {
    Pipeline* pl = (Pipeline*)handle;
    if (!pl) { g_err = "null pipeline"; return HIPBP_ERR_ARG; }
    std::lock_guard<std::mutex> lk(pl->e->mu);
    return pl->flush();
}

int hipbp_pipeline_prefix_tables(void* handle, int bits) {
    Pipeline* pl = (Pipeline*)handle;
    if (!pl) { g_err = "null pipeline"; return HIPBP_ERR_ARG; }
    if (bits < 0 || bits > bp::PREFIX_MAX_BITS) { g_err = "prefix bits must be 0..24"; return HIPBP_ERR_ARG; }
    std::lock_guard<std::mutex> lk(pl->e->mu);
    if (pl->busy()) { g_err = "prefix tables: pipeline has batches in flight (flush first)"; return HIPBP_ERR_ARG; }
    BP_RET_ON(hipStreamSynchronize(pl->s));
    pl->pbits = 0;
    pl->ext_tab = nullptr;
    if (pl->ptab.p) {
        BP_RET_ON(hipFree(pl->ptab.p));
        pl->ptab.p = nullptr;
        pl->ptab.cap = 0;
    }
    if (!bits) return HIPBP_OK;
    const size_t bytes = ((size_t)(2 * pl->n + 2) << bits) * sizeof(bp::ge);
    BP_RET_ON(pl->ptab.need(bytes));
    bp::launch_prefix_tables(pl->ptab.as<bp::ge>(), pl->G, pl->H, pl->h, pl->g, pl->n, bits, pl->s);
    BP_RET_ON(hipGetLastError());
    BP_RET_ON(hipStreamSynchronize(pl->s));
    pl->pbits = bits;
    return HIPBP_OK;
}

int hipbp_pipeline_depth(void* handle) { return handle ? ((Pipeline*)handle)->D : 0; }

void hipbp_pipeline_destroy(void* handle) {
    Pipeline* pl = (Pipeline*)handle;
    if (!pl) return;
    pl->release();
    delete pl;
}

int hipbp_msm(ge25519* result, const fe25519* scalars, const ge25519* points, size_t n, void* stream) {
    hipError_t err;
    Engine* e = engine_or_null(&err);
    BP_RET_ON(err);
    if (n == 0) return HIPBP_OK;
    if (!result || !scalars || !points) { g_err = "null argument"; return HIPBP_ERR_ARG; }
    std::lock_guard<std::mutex> lk(e->mu);
    hipStream_t s = pick(stream, *e);
    BP_RET_ON(msm_run(*e, (bp::ge*)result, (const bp::fe*)scalars, (const bp::ge*)points, n, 1, s));
    BP_RET_ON(hipGetLastError());
    return HIPBP_OK;
}

int hipbp_msm_batch(ge25519* results, const fe25519* scalars, const ge25519* points, size_t n, size_t count,
                    void* stream) {
    hipError_t err;
    Engine* e = engine_or_null(&err);
    BP_RET_ON(err);
    if (n == 0 || count == 0) return HIPBP_OK;
    if (!results || !scalars || !points) { g_err = "null argument"; return HIPBP_ERR_ARG; }
    if (count > 0x7FFFFFFFull || n * count > 0xFFFFFFFFull) { g_err = "msm_batch: too many items"; return HIPBP_ERR_ARG; }
    std::lock_guard<std::mutex> lk(e->mu);
    hipStream_t s = pick(stream, *e);
    BP_RET_ON(msm_run(*e, (bp::ge*)results, (const bp::fe*)scalars, (const bp::ge*)points, n, count, s));
    BP_RET_ON(hipGetLastError());
    return HIPBP_OK;
}

int hipbp_msm_batch_gens(ge25519* results, const fe25519* scalars, const void* gens, size_t count, void* stream) {
    hipError_t err;
    Engine* e = engine_or_null(&err);
    BP_RET_ON(err);
    const Gens* gs = (const Gens*)gens;
    if (!gs) { g_err = "null gens"; return HIPBP_ERR_ARG; }
    if (count == 0 || gs->n == 0) return HIPBP_OK;
    if (!results || !scalars) { g_err = "null argument"; return HIPBP_ERR_ARG; }
    if (gs->device != e->device) { g_err = "gens: created on another device"; return HIPBP_ERR_ARG; }
    const size_t n = 2 * gs->n;
    if (count > 0x7FFFFFFFull || n * count > 0xFFFFFFFFull) { g_err = "msm_batch_gens: too many items"; return HIPBP_ERR_ARG; }
    std::lock_guard<std::mutex> lk(e->mu);
    hipStream_t s = pick(stream, *e);
    BP_RET_ON(msm_run(*e, (bp::ge*)results, (const bp::fe*)scalars, gs->G(), n, count, s,
                      gs->bits ? gs->tab.as<bp::ge>() : nullptr, gs->bits));
    BP_RET_ON(hipGetLastError());
    return HIPBP_OK;
}

int hipbp_msm_pippenger_batch(ge25519* results, const fe25519* scalars, const ge25519* points, size_t n,
                              size_t count, int window_bits, void* stream) {
    hipError_t err;
    Engine* e = engine_or_null(&err);
    BP_RET_ON(err);
    if (n == 0 || count == 0) return HIPBP_OK;
    if (!results || !scalars || !points) { g_err = "null argument"; return HIPBP_ERR_ARG; }
    if (window_bits < 4 || window_bits > 12) { g_err = "pippenger: window_bits must be 4..12"; return HIPBP_ERR_ARG; }
    if (count > 0xFFFFu || n * count * ((256 + window_bits - 1) / window_bits) > 0x7FFFFFFFull) {
        g_err = "pippenger: n * count too large";
        return HIPBP_ERR_ARG;
    }
    std::lock_guard<std::mutex> lk(e->mu);
    BP_RET_ON(bp::msm_pippenger((bp::ge*)results, (const bp::fe*)scalars, (const bp::ge*)points, n, count, window_bits,
                                e->dtab, pick(stream, *e)));
    return HIPBP_OK;
}

int hipbp_msm_pippenger(ge25519* result, const fe25519* scalars, const ge25519* points, size_t n, int window_bits,
                        void* stream) {
    return hipbp_msm_pippenger_batch(result, scalars, points, n, 1, window_bits, stream);
}

int hipbp_msm_pippenger_windows(ge25519* window_sums, const fe25519* scalars, const ge25519* points, size_t n,
                                int window_bits, int w_begin, int w_end, void* stream) {
    hipError_t err;
    Engine* e = engine_or_null(&err);
    BP_RET_ON(err);
    if (window_bits < 4 || window_bits > 12) { g_err = "pippenger: window_bits must be 4..12"; return HIPBP_ERR_ARG; }
    const int W = (256 + window_bits - 1) / window_bits;
    if (w_begin < 0 || w_end > W || w_begin > w_end) { g_err = "pippenger_windows: need 0 <= w_begin <= w_end <= W"; return HIPBP_ERR_ARG; }
    if (n == 0 || w_begin == w_end) return HIPBP_OK;
    if (!window_sums || !scalars || !points) { g_err = "null argument"; return HIPBP_ERR_ARG; }
    if (n * (size_t)(w_end - w_begin) > 0x7FFFFFFFull) { g_err = "pippenger: n * windows too large"; return HIPBP_ERR_ARG; }
    std::lock_guard<std::mutex> lk(e->mu);
    BP_RET_ON(bp::msm_pippenger_windows((bp::ge*)window_sums, (const bp::fe*)scalars, (const bp::ge*)points, n,
                                        window_bits, w_begin, w_end, e->dtab, pick(stream, *e)));
    return HIPBP_OK;
}

// Frees every per-stream workspace the engine keeps for `stream` on the current device (canonical
// MSM / point-tree buffers, prover buffers, one-shot verify pipelines, Pippenger workspace pair),
// after waiting for the stream.  A later call on that stream builds them again.
int hipbp_release_stream_workspaces(void* stream) {
    hipError_t err;
    Engine* e = engine_or_null(&err);
    BP_RET_ON(err);
    hipStream_t s = (hipStream_t)stream;
    std::lock_guard<std::mutex> lk(e->mu);
    // every cached workspace of s is freed and its map entry removed even if a hipFree fails (no
    // pointer is left behind for a later call to reuse or free twice); the first error is returned
    hipError_t first = hipStreamSynchronize(s);
    auto keep = [&first](hipError_t r) { if (first == hipSuccess) first = r; };
    auto free_all = [&keep](Buf* bs, size_t nb) {
        for (size_t i = 0; i < nb; i++)
            if (bs[i].p) {
                keep(hipFree(bs[i].p));
                bs[i].p = nullptr;
                bs[i].cap = 0;
            }
    };
    auto mi = e->msm_ws.find(s);
    if (mi != e->msm_ws.end()) {
        free_all(mi->second->b, sizeof(mi->second->b) / sizeof(mi->second->b[0]));
        delete mi->second;
        e->msm_ws.erase(mi);
    }
    auto pi = e->provers.find(s);
    if (pi != e->provers.end()) {
        free_all(pi->second->b, sizeof(pi->second->b) / sizeof(pi->second->b[0]));
        delete pi->second;
        e->provers.erase(pi);
    }
    for (auto it = e->pipes.begin(); it != e->pipes.end();) {
        if (std::get<0>(it->first) == s) {
            it->second->release();
            delete it->second;
            it = e->pipes.erase(it);
        } else {
            ++it;
        }
    }
    keep(bp::pippenger_release(s));
    if (first != hipSuccess) {
        g_err = std::string("release_stream_workspaces: ") + hipGetErrorString(first);
        return HIPBP_ERR_DEVICE;
    }
    return HIPBP_OK;
}

int hipbp_msm_pippenger_horner(ge25519* results, const ge25519* window_sums, size_t count, int window_bits,
                               void* stream) {
    hipError_t err;
    Engine* e = engine_or_null(&err);
    BP_RET_ON(err);
    if (window_bits < 4 || window_bits > 12) { g_err = "pippenger: window_bits must be 4..12"; return HIPBP_ERR_ARG; }
    if (count == 0) return HIPBP_OK;
    if (!results || !window_sums) { g_err = "null argument"; return HIPBP_ERR_ARG; }
    if (count > 0xFFFFu) { g_err = "pippenger_horner: count <= 65535"; return HIPBP_ERR_ARG; }
    std::lock_guard<std::mutex> lk(e->mu);
    BP_RET_ON(bp::pippenger_horner((bp::ge*)results, (const bp::ge*)window_sums, count, window_bits,
                                   pick(stream, *e)));
    return HIPBP_OK;
}

static int prove_run(const hipbp_prove_input* in, const ge25519* G, const ge25519* H, const ge25519* g,
                     const ge25519* h, const bp::ge* ptab, int pbits, hipbp_proof_out* out, void* stream) {
    hipError_t err;
    Engine* e = engine_or_null(&err);
    BP_RET_ON(err);
    if (!in || !out || !G || !H || !g || !h) { g_err = "null argument"; return HIPBP_ERR_ARG; }
    if (in->count == 0) return HIPBP_OK;
    if (!is_pow2(in->n) || in->n > 128) { g_err = "prover: n must be a power of two <= 128"; return HIPBP_ERR_ARG; }
    if (in->count > ((size_t)1 << 22)) { g_err = "prover: batch too large"; return HIPBP_ERR_ARG; }
    if (!in->v || !in->gamma || !in->sL || !in->sR || !in->rnd) { g_err = "prover: null input"; return HIPBP_ERR_ARG; }
    if (!out->V || !out->A || !out->S || !out->T1 || !out->T2 || !out->taux || !out->mu || !out->t || !out->c ||
        !out->x || !out->a || !out->b || !out->valid || (in->n > 1 && (!out->L || !out->R))) {
        g_err = "prover: null output";
        return HIPBP_ERR_ARG;
    }
    std::lock_guard<std::mutex> lk(e->mu);
    BP_RET_ON(e->ensure_two((int)in->n));
    const size_t B = in->count, n = in->n;
    bp::ProveIn pin{(int)B, (int)n, log2i(n), (const bp::fe*)in->v, (const bp::fe*)in->gamma,
                    (const bp::fe*)in->sL, (const bp::fe*)in->sR, (const bp::fe*)in->rnd};
    bp::ProveOut po{(bp::ge*)out->V, (bp::ge*)out->A, (bp::ge*)out->S, (bp::ge*)out->T1, (bp::ge*)out->T2,
                    (bp::fe*)out->taux, (bp::fe*)out->mu, (bp::fe*)out->t, (bp::fe*)out->c, (bp::fe*)out->x,
                    (bp::fe*)out->a, (bp::fe*)out->b, (bp::ge*)out->L, (bp::ge*)out->R, out->valid};
    // workspace: prover buffers are the engine's prv[] (reused across calls on the engine's lock)
    const size_t FE = sizeof(bp::fe), GE = sizeof(bp::ge);
    const size_t cap = B * (4 * n + 4);
    size_t sz[17] = {B * 4 * n * FE, cap * GE, B * 4 * GE, B * 5 * GE, B * 8 * FE, B * 4 * FE, B * 4 * GE,
                     B * n * FE, B * n * FE, B * 2 * n * FE, B * 2 * FE, B * (2 * n + 2) * GE, B * 4 * FE, B,
                     2 * cap * sizeof(uint32_t), 2 * sizeof(unsigned), 2 * n * GE};
    hipStream_t s = pick(stream, *e);
    Engine::ProverBufs*& pb = e->provers[s];
    if (!pb) pb = new Engine::ProverBufs();
    Buf* prv = pb->b;
    // terms0's heavy-list sort (HIPBP_PROVE_SORT=0 turns it off, for A/B runs)
    static const bool psort = getenv("HIPBP_PROVE_SORT") ? atoi(getenv("HIPBP_PROVE_SORT")) != 0 : true;
    const int nbuf = psort ? 19 : 17;
    size_t sz2[19];
    for (int i = 0; i < 19; i++) sz2[i] = i < 17 ? sz[i] : 0;
    if (psort) { sz2[17] = cap * sizeof(uint32_t); sz2[18] = bp::MSM_BINS * sizeof(unsigned); }
    for (int i = 0; i < nbuf; i++) BP_RET_ON(prv[i].need(sz2[i]));
    bp::ProveWs w{prv[0].as<bp::fe>(), prv[1].as<bp::ge>(), prv[2].as<bp::ge>(), prv[3].as<bp::ge>(),
                  prv[4].as<bp::fe>(), prv[5].as<bp::fe>(), prv[6].as<bp::ge>(), prv[7].as<bp::fe>(),
                  prv[8].as<bp::fe>(), prv[9].as<bp::fe>(), prv[10].as<bp::fe>(), prv[11].as<bp::ge>(),
                  prv[12].as<bp::fe>(), prv[13].as<uint8_t>(), prv[14].as<uint32_t>(), prv[15].as<unsigned>(), cap,
                  prv[16].as<bp::ge>(), psort ? prv[17].as<uint32_t>() : nullptr,
                  psort ? prv[18].as<unsigned>() : nullptr, ptab, ptab ? pbits : 0};
    auto run = [&](int stage, int r) {
        bp::launch_prove(stage, r, pin, w, po, (const bp::ge*)G, (const bp::ge*)H, (const bp::ge*)g,
                         (const bp::ge*)h, e->dtab, e->two_i, s);
    };
    run(bp::PS_PREP, 0);
    run(bp::PS_SORT0, 0);
    run(bp::PS_TERMS0, 0);
    // the tail (chain0 .. final: ~20 short dependent launches) on the caller's stream; a side stream,
    // a terms0 gate across streams and other tail schedules were measured and rejected
    run(bp::PS_CHAIN0, 0);
    run(bp::PS_COMMIT, 0);
    run(bp::PS_TERMS1, 0);
    run(bp::PS_TX, 0);
    for (int r = 0; r < pin.L; r++) {
        run(bp::PS_RTERMS, r);
        run(bp::PS_RCHAIN, r);
        run(bp::PS_ROUND, r);
    }
    run(bp::PS_FINAL, 0);
    BP_RET_ON(hipGetLastError());
    return HIPBP_OK;
}

int hipbp_batch_generate_range_proof(const hipbp_prove_input* in, const ge25519* G, const ge25519* H,
                                     const ge25519* g, const ge25519* h, hipbp_proof_out* out, void* stream) {
    return prove_run(in, G, H, g, h, nullptr, 0, out, stream);
}

void* hipbp_gens_create(size_t n, const ge25519* G, const ge25519* H, const ge25519* g, const ge25519* h,
                        int prefix_bits, void* stream) {
    hipError_t err;
    Engine* e = engine_or_null(&err);
    if (!e) { g_err = std::string("engine: ") + hipGetErrorString(err); return nullptr; }
    if (!is_pow2(n) || n > MAX_N || !G || !H || !g || !h) { g_err = "gens: bad n or null generator"; return nullptr; }
    if (prefix_bits < 0 || prefix_bits > bp::PREFIX_MAX_BITS) { g_err = "gens: prefix bits must be 0..24"; return nullptr; }
    Gens* gs = new Gens();
    gs->device = e->device;
    gs->n = n;
    hipStream_t s = pick(stream, *e);
    const size_t GE = sizeof(ge25519);
    auto fail = [&](hipError_t er, const char* what) -> void* {
        g_err = std::string(what) + ": " + hipGetErrorString(er);
        gs->release();
        delete gs;
        return nullptr;
    };
    if ((err = gs->gen.need((2 * n + 2) * GE)) != hipSuccess) return fail(err, "gens alloc");
    uint8_t* d = gs->gen.as<uint8_t>();   // snapshot: G | H | h | g (the table base order)
    if ((err = hipMemcpyAsync(d, G, n * GE, hipMemcpyDeviceToDevice, s)) != hipSuccess) return fail(err, "gens copy");
    if ((err = hipMemcpyAsync(d + n * GE, H, n * GE, hipMemcpyDeviceToDevice, s)) != hipSuccess) return fail(err, "gens copy");
    if ((err = hipMemcpyAsync(d + 2 * n * GE, h, GE, hipMemcpyDeviceToDevice, s)) != hipSuccess) return fail(err, "gens copy");
    if ((err = hipMemcpyAsync(d + (2 * n + 1) * GE, g, GE, hipMemcpyDeviceToDevice, s)) != hipSuccess)
        return fail(err, "gens copy");
    if (prefix_bits) {
        if ((err = gs->tab.need(((2 * n + 2) << prefix_bits) * GE)) != hipSuccess) return fail(err, "gens tables");
        bp::launch_prefix_tables(gs->tab.as<bp::ge>(), gs->G(), gs->H(), gs->h(), gs->g(), (int)n, prefix_bits, s);
        if ((err = hipGetLastError()) != hipSuccess) return fail(err, "gens tables");
        gs->bits = prefix_bits;
    }
    if ((err = hipStreamSynchronize(s)) != hipSuccess) return fail(err, "gens sync");
    return gs;
}

void hipbp_gens_destroy(void* gens) {
    Gens* gs = (Gens*)gens;
    if (!gs) return;
    gs->release();
    delete gs;
}

int hipbp_batch_generate_range_proof_gens(const hipbp_prove_input* in, void* gens, hipbp_proof_out* out,
                                          void* stream) {
    Gens* gs = (Gens*)gens;
    if (!gs) { g_err = "null gens"; return HIPBP_ERR_ARG; }
    if (!in || in->n != gs->n) { g_err = "prover: input n differs from the generator set's"; return HIPBP_ERR_ARG; }
    int dev = -1;
    BP_RET_ON(hipGetDevice(&dev));
    if (dev != gs->device) { g_err = "gens: created on another device"; return HIPBP_ERR_ARG; }
    return prove_run(in, (const ge25519*)gs->G(), (const ge25519*)gs->H(), (const ge25519*)gs->g(),
                     (const ge25519*)gs->h(), gs->bits ? gs->tab.as<bp::ge>() : nullptr, gs->bits, out, stream);
}

int hipbp_pipeline_use_gens(void* handle, void* gens) {
    Pipeline* pl = (Pipeline*)handle;
    Gens* gs = (Gens*)gens;
    if (!pl || !gs) { g_err = "null pipeline or gens"; return HIPBP_ERR_ARG; }
    if ((int)gs->n != pl->n) { g_err = "pipeline n differs from the generator set's"; return HIPBP_ERR_ARG; }
    if (gs->device != pl->e->device) { g_err = "gens: created on another device"; return HIPBP_ERR_ARG; }
    std::lock_guard<std::mutex> lk(pl->e->mu);
    if (pl->busy()) { g_err = "use_gens: pipeline has batches in flight (flush first)"; return HIPBP_ERR_ARG; }
    BP_RET_ON(hipStreamSynchronize(pl->s));
    if (pl->ptab.p) {   // its own tables (hipbp_pipeline_prefix_tables) give way to the set's
        BP_RET_ON(hipFree(pl->ptab.p));
        pl->ptab.p = nullptr;
        pl->ptab.cap = 0;
    }
    pl->G = gs->G();
    pl->H = gs->H();
    pl->h = gs->h();
    pl->g = gs->g();
    pl->ext_tab = gs->bits ? gs->tab.as<bp::ge>() : nullptr;
    pl->pbits = gs->bits;
    return HIPBP_OK;
}

int hipbp_pipeline_defer_msm(void* handle, int on) {
    Pipeline* pl = (Pipeline*)handle;
    if (!pl) { g_err = "null pipeline"; return HIPBP_ERR_ARG; }
    if (on && !pl->defer_ok()) {
        g_err = "defer_msm: needs cuda_range_proof_verify / range_proof_verify semantics, 4 <= n <= the lane-tree limit "
                "and n <= 512 (a split tick's region list)";
        return HIPBP_ERR_ARG;
    }
    std::lock_guard<std::mutex> lk(pl->e->mu);
    pl->defer_msm = on != 0;   // applies to the batches pushed from now on
    return HIPBP_OK;
}

int hipbp_point_tree(ge25519* result, const ge25519* points, size_t n, void* stream) {
    hipError_t err;
    Engine* e = engine_or_null(&err);
    BP_RET_ON(err);
    if (n == 0) return HIPBP_OK;
    if (!result || !points) { g_err = "null argument"; return HIPBP_ERR_ARG; }
    std::lock_guard<std::mutex> lk(e->mu);
    size_t nb = (n + 255) / 256;
    hipStream_t s = pick(stream, *e);
    Buf* w = e->msm_bufs(s);
    BP_RET_ON(w[3].need(nb * sizeof(bp::ge)));
    BP_RET_ON(w[4].need(nb * sizeof(bp::ge)));
    bp::launch_tree_full((bp::ge*)result, (const bp::ge*)points, n, w[3].as<bp::ge>(), w[4].as<bp::ge>(), s);
    BP_RET_ON(hipGetLastError());
    return HIPBP_OK;
}

int hipbp_field_op(int op, fe25519* r, const fe25519* a, const fe25519* b, size_t count, void* stream) {
    hipError_t err;
    Engine* e = engine_or_null(&err);
    BP_RET_ON(err);
    if (op < 0 || op > 20) { g_err = "bad op"; return HIPBP_ERR_ARG; }
    if (!a || (!b && op != 3 && op != 5 && op != 7 && op != 11 && op != 12)) { g_err = "null operand"; return HIPBP_ERR_ARG; }
    if (count == 0) return HIPBP_OK;
    hipStream_t s = pick(stream, *e);
    if (op == 5)
        bp::launch_invert((bp::fe*)r, (const bp::fe*)a, count, s);
    else
        bp::launch_field_op(op, (bp::fe*)r, (const bp::fe*)a, (const bp::fe*)b, count, s);
    BP_RET_ON(hipGetLastError());
    return HIPBP_OK;
}

int hipbp_sha_probe(int kind, fe25519* out, const fe25519* in, size_t count, void* stream) {
    hipError_t err;
    Engine* e = engine_or_null(&err);
    BP_RET_ON(err);
    if (kind < 0 || kind > 5) { g_err = "bad sha probe kind"; return HIPBP_ERR_ARG; }
    if (!out || !in) { g_err = "null operand"; return HIPBP_ERR_ARG; }
    if (count == 0) return HIPBP_OK;
    bp::launch_sha_probe(kind, (bp::fe*)out, (const bp::fe*)in, count, pick(stream, *e));
    BP_RET_ON(hipGetLastError());
    return HIPBP_OK;
}

// ===================================================================== reference surface

void cuda_point_vector_multi_scalar_mul(ge25519* result, const FieldVector* scalars, const PointVector* points) {
    if (scalars->length != points->length) {   // cuda_bulletproof_kernels.cu:65-68
        fprintf(stderr, "Error: Vector lengths must match for multi-scalar multiplication\n");
        return;
    }
    size_t n = scalars->length;
    if (n == 0) return;
    Engine& e = engine_or_exit();
    std::lock_guard<std::mutex> lk(e.mu);
    BP_EXIT_ON(e.h2d[0].need(n * sizeof(fe25519)));
    BP_EXIT_ON(e.h2d[1].need(n * sizeof(ge25519)));
    BP_EXIT_ON(e.h2d[2].need(sizeof(ge25519)));
    BP_EXIT_ON(hipMemcpyAsync(e.h2d[0].p, scalars->elements, n * sizeof(fe25519), hipMemcpyHostToDevice, e.stream));
    BP_EXIT_ON(hipMemcpyAsync(e.h2d[1].p, points->elements, n * sizeof(ge25519), hipMemcpyHostToDevice, e.stream));
    BP_EXIT_ON(msm_run(e, e.h2d[2].as<bp::ge>(), e.h2d[0].as<bp::fe>(), e.h2d[1].as<bp::ge>(), n, 1, e.stream));
    BP_EXIT_ON(hipMemcpyAsync(result, e.h2d[2].p, sizeof(ge25519), hipMemcpyDeviceToHost, e.stream));
    BP_EXIT_ON(hipStreamSynchronize(e.stream));
}

void cuda_point_vector_multi_scalar_mul_shared(ge25519* result, const FieldVector* scalars,
                                               const PointVector* points) {
    // cuda_bulletproof_kernels.cu:119-138: the n <= 64 shared-memory kernel computes the
    // same canonical tree; larger n delegates to the standard path.
    cuda_point_vector_multi_scalar_mul(result, scalars, points);
}

static void ip_common(fe25519* result, const FieldVector* a, const FieldVector* b, bool force_shared) {
    if (a->length != b->length) {   // cuda_inner_product.cu:100-103
        fprintf(stderr, "Error: Vector lengths must match for inner product\n");
        return;
    }
    size_t n = a->length;
    if (n == 0) return;
    Engine& e = engine_or_exit();
    std::lock_guard<std::mutex> lk(e.mu);
    BP_EXIT_ON(e.h2d[0].need(n * sizeof(fe25519)));
    BP_EXIT_ON(e.h2d[1].need(n * sizeof(fe25519)));
    BP_EXIT_ON(e.h2d[2].need(sizeof(fe25519)));
    BP_EXIT_ON(e.scratch[3].need(1024 * sizeof(fe25519)));
    BP_EXIT_ON(hipMemcpyAsync(e.h2d[0].p, a->elements, n * sizeof(fe25519), hipMemcpyHostToDevice, e.stream));
    BP_EXIT_ON(hipMemcpyAsync(e.h2d[1].p, b->elements, n * sizeof(fe25519), hipMemcpyHostToDevice, e.stream));
    if (force_shared || n <= 512)
        bp::launch_ip_shared(e.h2d[2].as<bp::fe>(), e.h2d[0].as<bp::fe>(), e.h2d[1].as<bp::fe>(), n, e.stream);
    else
        bp::launch_ip_grid(e.h2d[2].as<bp::fe>(), e.scratch[3].as<bp::fe>(), e.h2d[0].as<bp::fe>(),
                           e.h2d[1].as<bp::fe>(), n, e.stream);
    BP_EXIT_ON(hipGetLastError());
    BP_EXIT_ON(hipMemcpyAsync(result, e.h2d[2].p, sizeof(fe25519), hipMemcpyDeviceToHost, e.stream));
    BP_EXIT_ON(hipStreamSynchronize(e.stream));
}

void cuda_field_vector_inner_product(fe25519* result, const FieldVector* a, const FieldVector* b) {
    ip_common(result, a, b, false);
}

void cuda_field_vector_inner_product_shared(fe25519* result, const FieldVector* a, const FieldVector* b) {
    ip_common(result, a, b, true);
}

void cuda_batch_field_vector_inner_product(fe25519* results, const FieldVector* a_vectors,
                                           const FieldVector* b_vectors, size_t num_vectors) {
    if (num_vectors == 0) return;
    size_t n = a_vectors[0].length;   // cuda_inner_product.cu:306: every vector taken at vector 0's length
    Engine& e = engine_or_exit();
    std::lock_guard<std::mutex> lk(e.mu);
    size_t tot = num_vectors * n;
    BP_EXIT_ON(e.h2d[0].need(tot * sizeof(fe25519) + 32));
    BP_EXIT_ON(e.h2d[1].need(tot * sizeof(fe25519) + 32));
    BP_EXIT_ON(e.h2d[2].need(num_vectors * sizeof(fe25519)));
    for (size_t i = 0; i < num_vectors; i++) {
        BP_EXIT_ON(hipMemcpyAsync(e.h2d[0].as<fe25519>() + i * n, a_vectors[i].elements, n * sizeof(fe25519),
                                  hipMemcpyHostToDevice, e.stream));
        BP_EXIT_ON(hipMemcpyAsync(e.h2d[1].as<fe25519>() + i * n, b_vectors[i].elements, n * sizeof(fe25519),
                                  hipMemcpyHostToDevice, e.stream));
    }
    bp::launch_ip_batch(e.h2d[2].as<bp::fe>(), e.h2d[0].as<bp::fe>(), e.h2d[1].as<bp::fe>(), n, num_vectors, e.stream);
    BP_EXIT_ON(hipGetLastError());
    BP_EXIT_ON(hipMemcpyAsync(results, e.h2d[2].p, num_vectors * sizeof(fe25519), hipMemcpyDeviceToHost, e.stream));
    BP_EXIT_ON(hipStreamSynchronize(e.stream));
}

static void field_common(int op, fe25519* results, const fe25519* a, const fe25519* b, size_t count) {
    if (count == 0) return;
    Engine& e = engine_or_exit();
    std::lock_guard<std::mutex> lk(e.mu);
    BP_EXIT_ON(e.h2d[0].need(count * sizeof(fe25519)));
    BP_EXIT_ON(e.h2d[1].need(count * sizeof(fe25519)));
    BP_EXIT_ON(e.h2d[2].need(count * sizeof(fe25519)));
    BP_EXIT_ON(hipMemcpyAsync(e.h2d[0].p, a, count * sizeof(fe25519), hipMemcpyHostToDevice, e.stream));
    if (b) BP_EXIT_ON(hipMemcpyAsync(e.h2d[1].p, b, count * sizeof(fe25519), hipMemcpyHostToDevice, e.stream));
    if (op == 5)
        bp::launch_invert(e.h2d[2].as<bp::fe>(), e.h2d[0].as<bp::fe>(), count, e.stream);
    else
        bp::launch_field_op(op, e.h2d[2].as<bp::fe>(), e.h2d[0].as<bp::fe>(), e.h2d[1].as<bp::fe>(), count, e.stream);
    BP_EXIT_ON(hipGetLastError());
    BP_EXIT_ON(hipMemcpyAsync(results, e.h2d[2].p, count * sizeof(fe25519), hipMemcpyDeviceToHost, e.stream));
    BP_EXIT_ON(hipStreamSynchronize(e.stream));
}

void cuda_batch_field_add(fe25519* r, const fe25519* a, const fe25519* b, size_t count) { field_common(0, r, a, b, count); }
void cuda_batch_field_sub(fe25519* r, const fe25519* a, const fe25519* b, size_t count) { field_common(1, r, a, b, count); }
void cuda_batch_field_mul(fe25519* r, const fe25519* a, const fe25519* b, size_t count) { field_common(2, r, a, b, count); }
void cuda_batch_field_mul_karatsuba(fe25519* r, const fe25519* a, const fe25519* b, size_t count) {
    field_common(2, r, a, b, count);   // cuda_field_ops.cu:73: schoolbook + the same fold == fe25519_mul
}
void cuda_batch_field_square(fe25519* r, const fe25519* in, size_t count) { field_common(3, r, in, nullptr, count); }
void cuda_batch_field_invert(fe25519* r, const fe25519* in, size_t count) { field_common(5, r, in, nullptr, count); }
void cuda_soa_field_add(fe25519* r, const fe25519* a, const fe25519* b, size_t count) { field_common(4, r, a, b, count); }

// Stage one proof (host structs) into the engine's device staging buffers as a batch of 1.
static bool stage_single(Engine& e, const InnerProductProof* ip, const RangeProof* rp, const ge25519* V,
                         hipbp_proof_batch* b) {
    size_t abl = ip->a.length, Lr = ip->L_len;
    if (ip->b.length != abl || abl == 0 || ip->L.length < Lr || ip->R.length < Lr) return false;
    // head: V,A,S,T1,T2 | t,c,x ; then a,b ; then L,R
    size_t bytes = 5 * sizeof(ge25519) + 3 * sizeof(fe25519) + 2 * abl * sizeof(fe25519) + 2 * Lr * sizeof(ge25519);
    BP_EXIT_ON(e.h2d[3].need(bytes));
    BP_EXIT_ON(e.need_pinned(bytes));
    BP_EXIT_ON(hipStreamSynchronize(e.stream));   // previous user of the staging buffer is done
    uint8_t* q = e.pinned;
    auto put = [&](const void* src, size_t len) {
        if (src) memcpy(q, src, len);
        else memset(q, 0, len);
        q += len;
    };
    const ge25519 zero_pt = {};
    put(V ? V : &zero_pt, sizeof(ge25519));
    put(rp ? &rp->A : nullptr, sizeof(ge25519));
    put(rp ? &rp->S : nullptr, sizeof(ge25519));
    put(rp ? &rp->T1 : nullptr, sizeof(ge25519));
    put(rp ? &rp->T2 : nullptr, sizeof(ge25519));
    put(rp ? &rp->t : nullptr, sizeof(fe25519));
    put(&ip->c, sizeof(fe25519));
    put(&ip->x, sizeof(fe25519));
    put(ip->a.elements, abl * sizeof(fe25519));
    put(ip->b.elements, abl * sizeof(fe25519));
    if (Lr) {
        put(ip->L.elements, Lr * sizeof(ge25519));
        put(ip->R.elements, Lr * sizeof(ge25519));
    }
    BP_EXIT_ON(hipMemcpyAsync(e.h2d[3].p, e.pinned, bytes, hipMemcpyHostToDevice, e.stream));
    uint8_t* d = e.h2d[3].as<uint8_t>();
    const ge25519* pts = (const ge25519*)d;
    const fe25519* fes = (const fe25519*)(d + 5 * sizeof(ge25519));
    b->count = 1;
    b->ab_len = abl;
    b->L_len = Lr;
    b->V = pts + 0; b->A = pts + 1; b->S = pts + 2; b->T1 = pts + 3; b->T2 = pts + 4;
    b->t = fes + 0; b->c = fes + 1; b->x = fes + 2;
    b->a = fes + 3;
    b->b = fes + 3 + abl;
    const ge25519* lr = (const ge25519*)(d + 5 * sizeof(ge25519) + (3 + 2 * abl) * sizeof(fe25519));
    b->L = Lr ? lr : nullptr;
    b->R = Lr ? lr + Lr : nullptr;
    return true;
}

static bool verify_single(const InnerProductProof* ip, const RangeProof* rp, const ge25519* V, const ge25519* P,
                          size_t n, const PointVector* G, const PointVector* H, const ge25519* h) {
    Engine& e = engine_or_exit();
    std::lock_guard<std::mutex> lk(e.mu);
    hipbp_proof_batch b;
    memset(&b, 0, sizeof b);
    if (!stage_single(e, ip, rp, V, &b)) return false;
    b.n = n;
    // generators + h + P
    const size_t cap0 = e.h2d[4].cap;
    BP_EXIT_ON(e.h2d[4].need(2 * n * sizeof(ge25519) + 3 * sizeof(ge25519)));
    if (e.h2d[4].cap != cap0) e.single_gens.clear();   // a new buffer (maybe at the old address) holds nothing
    ge25519* dg = e.h2d[4].as<ge25519>();
    const size_t GB = n * sizeof(ge25519);
    std::vector<uint8_t>& sg = e.single_gens;
    const bool same = e.single_gens_dev == (const void*)dg && sg.size() == 2 * GB + sizeof(ge25519) &&
                      memcmp(sg.data(), G->elements, GB) == 0 && memcmp(sg.data() + GB, H->elements, GB) == 0 &&
                      memcmp(sg.data() + 2 * GB, h, sizeof(ge25519)) == 0;
    if (!same) {   // (every earlier user of dg has finished: each call ends with a stream sync)
        BP_EXIT_ON(hipMemcpyAsync(dg, G->elements, GB, hipMemcpyHostToDevice, e.stream));
        BP_EXIT_ON(hipMemcpyAsync(dg + n, H->elements, GB, hipMemcpyHostToDevice, e.stream));
        BP_EXIT_ON(hipMemcpyAsync(dg + 2 * n, h, sizeof(ge25519), hipMemcpyHostToDevice, e.stream));
        sg.resize(2 * GB + sizeof(ge25519));
        memcpy(sg.data(), G->elements, GB);
        memcpy(sg.data() + GB, H->elements, GB);
        memcpy(sg.data() + 2 * GB, h, sizeof(ge25519));
        e.single_gens_dev = dg;
    }
    if (P) BP_EXIT_ON(hipMemcpyAsync(dg + 2 * n + 1, P, sizeof(ge25519), hipMemcpyHostToDevice, e.stream));
    BP_EXIT_ON(e.h2d[5].need(64));
    int rc = run_verify(e, &b, P ? dg + 2 * n + 1 : nullptr, dg, dg + n, dg + 2 * n, e.h2d[5].as<uint8_t>(), nullptr,
                        nullptr, rp != nullptr ? 1 : 0, e.stream);
    if (rc == HIPBP_ERR_ARG) {
        fprintf(stderr, "Error: %s\n", g_err.c_str());
        return false;
    }
    if (rc != HIPBP_OK) {
        fprintf(stderr, "HIP error - %s\n", g_err.c_str());
        exit(EXIT_FAILURE);
    }
    uint8_t ok = 0;
    BP_EXIT_ON(hipMemcpyAsync(&ok, e.h2d[5].p, 1, hipMemcpyDeviceToHost, e.stream));
    BP_EXIT_ON(hipStreamSynchronize(e.stream));
    return ok != 0;
}

bool cuda_range_proof_verify(const RangeProof* proof, const ge25519* V, size_t n, const PointVector* G,
                             const PointVector* H, const ge25519* g, const ge25519* h) {
    (void)g;
    const InnerProductProof* ip = &proof->ip_proof;
    if (G->length != ip->n || H->length != ip->n || n != ip->n) {   // crv:140-143 (and rp.cu:658 reads n entries)
        fprintf(stderr, "Error: Vector lengths must match for inner product verification\n");
        return false;
    }
    return verify_single(ip, proof, V, nullptr, n, G, H, h);
}

bool cuda_inner_product_verify(const InnerProductProof* proof, const ge25519* P, const PointVector* G,
                               const PointVector* H, const ge25519* Q) {
    if (G->length != proof->n || H->length != proof->n) {   // crv:140-143
        fprintf(stderr, "Error: Vector lengths must match for inner product verification\n");
        return false;
    }
    return verify_single(proof, nullptr, nullptr, P, proof->n, G, H, Q);
}

// ---- batch form of cuda_range_proof_verify over the reference's host RangeProof structs
}  // extern "C"

namespace {

// one device's shard of hipbp_batch_range_proof_verify_host (its own host thread).  The shard is cut
// into chunks of CHUNK proofs, each staged as its own little flat batch; each chunk is packed,
// copied and pushed as soon as it is packed (the GPU starts while the host packs the rest), and
// the chunks alternate over two pipelines on two streams, whose ticks fill each other's tails.
int host_shard(int dev, const RangeProof* proofs, const ge25519* V, const size_t* idx, size_t B, size_t abl,
               size_t Lr, size_t n, const PointVector* G, const PointVector* H, const ge25519* h, uint8_t* ok) {
    BP_RET_ON(hipSetDevice(dev));
    hipError_t err;
    Engine* e = engine_or_null(&err);
    BP_RET_ON(err);
    constexpr size_t CHUNK = 1024;
    const size_t GE = sizeof(ge25519), FE = sizeof(fe25519);
    // per chunk of c proofs: V A S T1 T2 [c] | t c x [c] | a b [c abl] | L R [c Lr]
    auto chunk_bytes = [&](size_t c) { return c * (5 * GE + 3 * FE + 2 * abl * FE + 2 * Lr * GE); };
    const size_t nch = (B + CHUNK - 1) / CHUNK;
    const size_t gen_off = chunk_bytes(CHUNK) * (nch - 1) + chunk_bytes(B - CHUNK * (nch - 1));
    const size_t ok_off = gen_off + (2 * n + 1) * GE, bytes = ok_off + B;
    std::lock_guard<std::mutex> lk(e->mu);
    if (!e->stream2) BP_RET_ON(hipStreamCreateWithFlags(&e->stream2, hipStreamNonBlocking));
    hipStream_t st[2] = {e->stream, e->stream2};
    if (bytes > e->host_pinned_cap) {
        if (e->host_pinned) {
            BP_RET_ON(hipStreamSynchronize(st[0]));
            BP_RET_ON(hipStreamSynchronize(st[1]));
            BP_RET_ON(hipHostFree(e->host_pinned));
            e->host_pinned = nullptr;
            e->host_pinned_cap = 0;
        }
        BP_RET_ON(hipHostMalloc((void**)&e->host_pinned, bytes));
        e->host_pinned_cap = bytes;
    }
    if (bytes > e->host_dev.cap) {   // Buf::need frees the old buffer: nothing may still read it
        BP_RET_ON(hipStreamSynchronize(st[0]));
        BP_RET_ON(hipStreamSynchronize(st[1]));
    }
    BP_RET_ON(e->host_dev.need(bytes));
    uint8_t* host = e->host_pinned;
    uint8_t* dbuf = e->host_dev.as<uint8_t>();
    memcpy(host + gen_off, G->elements, n * GE);
    memcpy(host + gen_off + n * GE, H->elements, n * GE);
    memcpy(host + gen_off + 2 * n * GE, h, GE);
    BP_RET_ON(hipMemcpyAsync(dbuf + gen_off, host + gen_off, (2 * n + 1) * GE, hipMemcpyHostToDevice, st[0]));
    BP_RET_ON(e->ensure_two((int)n));   // engine stream: ordered before the pipeline's first tick
    const ge25519* dgen = (const ge25519*)(dbuf + gen_off);
    // the generators' prefix tables: reused when this call's generator bytes equal the cached set's
    // (then the pipelines read this call's copy and the tables built from identical bytes)
    int hb = 16;
    if (const char* pb = getenv("HIPBP_HOST_PREFIX_BITS")) hb = std::max(0, std::min(atoi(pb), bp::PREFIX_MAX_BITS));
    while (hb > 0 && ((2 * n + 2) << hb) * GE > (size_t(5) << 28)) hb--;   // at most 1.25 GB of tables (K = 12 at n = 1024)
    if (hb > 0) {
        const uint8_t* key = host + gen_off;
        const size_t kb = (2 * n + 1) * GE;
        if (e->host_tab_bits != hb || e->host_gens_key.size() != kb || memcmp(e->host_gens_key.data(), key, kb) != 0) {
            e->host_tab_bits = 0;
            e->host_gens_key.clear();
            BP_RET_ON(hipStreamSynchronize(st[0]));   // a previous call's tables are no longer read
            BP_RET_ON(hipStreamSynchronize(st[1]));
            if (e->host_gens.need((2 * n + 2) * GE) != hipSuccess || e->host_tab.need(((2 * n + 2) << hb) * GE) != hipSuccess) {
                (void)hipGetLastError();   // no room for the tables: verify without them
                hb = 0;
            }
        }
        if (hb > 0 && e->host_tab_bits == 0) {
            uint8_t* dg = e->host_gens.as<uint8_t>();
            BP_RET_ON(hipMemcpyAsync(dg, dbuf + gen_off, kb, hipMemcpyDeviceToDevice, st[0]));
            BP_RET_ON(hipMemcpyAsync(dg + kb, dbuf + gen_off + 2 * n * GE, GE, hipMemcpyDeviceToDevice, st[0]));
            const bp::ge* gg = e->host_gens.as<bp::ge>();
            bp::launch_prefix_tables(e->host_tab.as<bp::ge>(), gg, gg + n, gg + 2 * n, gg + 2 * n + 1, (int)n, hb,
                                     st[0]);
            BP_RET_ON(hipGetLastError());
            e->host_gens_key.assign(key, key + kb);
            e->host_tab_bits = hb;
        }
    }
    Pipeline* pl[2] = {nullptr, nullptr};
    int rc = HIPBP_OK;
    for (int k = 0; k < 2 && rc == HIPBP_OK; k++) {
        rc = pipeline_for(*e, st[k], std::min(B, CHUNK), (int)n, 1, &pl[k]);
        if (rc == HIPBP_OK) {
            pl[k]->G = (const bp::ge*)dgen;
            pl[k]->H = (const bp::ge*)(dgen + n);
            pl[k]->h = (const bp::ge*)(dgen + 2 * n);
            pl[k]->g = nullptr;
            // (the engine's one-shot pipelines are shared with the other entry points: the tables
            // are lent for this call only and taken back after the flush below)
            pl[k]->ext_tab = hb > 0 ? e->host_tab.as<bp::ge>() : nullptr;
            pl[k]->pbits = hb > 0 ? hb : 0;
        }
    }
    hipEvent_t gens_ready = nullptr;
    if (rc == HIPBP_OK) {   // the second stream waits for the generators' copy
        BP_RET_ON(hipEventCreateWithFlags(&gens_ready, hipEventDisableTiming));
        BP_RET_ON(hipEventRecord(gens_ready, st[0]));
        BP_RET_ON(hipStreamWaitEvent(st[1], gens_ready, 0));
    }
    uint8_t* dok = dbuf + ok_off;
    size_t off = 0;
    for (size_t ch = 0; ch < nch && rc == HIPBP_OK; ch++) {
        const size_t c0 = ch * CHUNK, c = std::min(CHUNK, B - c0), cb = chunk_bytes(c);
        uint8_t* hc = host + off;
        ge25519* hg = (ge25519*)hc;
        fe25519* hf = (fe25519*)(hc + 5 * c * GE);
        fe25519* hab = hf + 3 * c;
        ge25519* hlr = (ge25519*)(hab + 2 * c * abl);
        for (size_t k = 0; k < c; k++) {
            const RangeProof& p = proofs[idx[c0 + k]];
            const InnerProductProof& ip = p.ip_proof;
            hg[k] = V[idx[c0 + k]];
            hg[c + k] = p.A;
            hg[2 * c + k] = p.S;
            hg[3 * c + k] = p.T1;
            hg[4 * c + k] = p.T2;
            hf[k] = p.t;
            hf[c + k] = ip.c;
            hf[2 * c + k] = ip.x;
            memcpy(hab + k * abl, ip.a.elements, abl * FE);
            memcpy(hab + (c + k) * abl, ip.b.elements, abl * FE);
            if (Lr) {
                memcpy(hlr + k * Lr, ip.L.elements, Lr * GE);
                memcpy(hlr + (c + k) * Lr, ip.R.elements, Lr * GE);
            }
        }
        hipStream_t s = st[ch & 1];
        if ((err = hipMemcpyAsync(dbuf + off, hc, cb, hipMemcpyHostToDevice, s)) != hipSuccess) {
            g_err = std::string("chunk H2D: ") + hipGetErrorString(err);
            rc = HIPBP_ERR_DEVICE;
            break;
        }
        const uint8_t* dc = dbuf + off;
        const ge25519* dg = (const ge25519*)dc;
        const fe25519* df = (const fe25519*)(dc + 5 * c * GE);
        hipbp_proof_batch b;
        memset(&b, 0, sizeof b);
        b.count = c;
        b.n = n;
        b.ab_len = abl;
        b.L_len = Lr;
        b.V = dg; b.A = dg + c; b.S = dg + 2 * c; b.T1 = dg + 3 * c; b.T2 = dg + 4 * c;
        b.t = df; b.c = df + c; b.x = df + 2 * c;
        b.a = df + 3 * c; b.b = df + 3 * c + c * abl;
        const ge25519* dlr = (const ge25519*)(df + 3 * c + 2 * c * abl);
        b.L = Lr ? dlr : nullptr;
        b.R = Lr ? dlr + c * Lr : nullptr;
        rc = pl[ch & 1]->push(&b, nullptr, dok + c0, nullptr, nullptr);
        off += cb;
    }
    for (int k = 0; k < 2 && rc == HIPBP_OK; k++) rc = pl[k]->flush();
    for (int k = 0; k < 2; k++)
        if (pl[k]) {
            pl[k]->ext_tab = nullptr;
            pl[k]->pbits = 0;
        }
    hipError_t s1 = hipStreamSynchronize(st[1]);
    if (rc == HIPBP_OK && s1 == hipSuccess) {
        if ((err = hipMemcpyAsync(host + ok_off, dok, B, hipMemcpyDeviceToHost, st[0])) == hipSuccess)
            err = hipStreamSynchronize(st[0]);
        if (err != hipSuccess) { g_err = std::string("shard D2H: ") + hipGetErrorString(err); rc = HIPBP_ERR_DEVICE; }
    } else {
        (void)hipStreamSynchronize(st[0]);   // nothing in flight reads the staging any more
        if (rc == HIPBP_OK) { g_err = std::string("stream2: ") + hipGetErrorString(s1); rc = HIPBP_ERR_DEVICE; }
    }
    if (gens_ready) (void)hipEventDestroy(gens_ready);
    if (rc == HIPBP_OK)
        for (size_t k = 0; k < B; k++) ok[idx[k]] = host[ok_off + k] ? 1 : 0;
    return rc;
}

}  // namespace

extern "C" {

int hipbp_batch_range_proof_verify_host(const RangeProof* proofs, const ge25519* V, size_t count, size_t n,
                                        const PointVector* G, const PointVector* H, const ge25519* g,
                                        const ge25519* h, int num_gpus, uint8_t* ok) {
    (void)g;   // g is not read by cuda_range_proof_verify (crv:82-127)
    if (count == 0) return HIPBP_OK;
    if (!proofs || !V || !G || !H || !h || !ok || !G->elements || !H->elements) {
        g_err = "null argument";
        return HIPBP_ERR_ARG;
    }
    int ndev = 0;
    BP_RET_ON(hipGetDeviceCount(&ndev));
    if (ndev <= 0) { g_err = "no HIP device"; return HIPBP_ERR_DEVICE; }
    if (num_gpus > ndev) {   // asked for more devices than are visible: an error, not a silent fallback
        g_err = "num_gpus = " + std::to_string(num_gpus) + " but " + std::to_string(ndev) + " HIP device(s) visible";
        return HIPBP_ERR_ARG;
    }
    int ng = num_gpus <= 0 ? ndev : num_gpus;
    // HIPBP_HOST_SHARDS=k (tests, only when the caller leaves num_gpus <= 0): k shards (at most 64
    // and at most one per proof), shard d on device (current + d) % ndev, so the multi-device split, its host
    // threads and the verdict merge also run on a one-GPU box (threads of one device serialise on
    // its engine's mutex)
    if (num_gpus <= 0)
        if (const char* hs = getenv("HIPBP_HOST_SHARDS"))
            if (atoi(hs) > 0) ng = (int)std::min<size_t>(std::min(atoi(hs), 64), std::max<size_t>(count, 1));
    // The flat batch needs one (a/b length, rounds) shape: the first proof that passes the checks
    // sets it (the reference prover's proofs all share it); proofs of another shape go one by one.
    size_t abl = 0, Lr = 0;
    std::vector<size_t> main, other;
    main.reserve(count);
    for (size_t i = 0; i < count; i++) {
        const InnerProductProof& ip = proofs[i].ip_proof;
        ok[i] = 0;
        if (G->length != ip.n || H->length != ip.n || n != ip.n) {   // crv:140-143, as the single call
            fprintf(stderr, "Error: Vector lengths must match for inner product verification\n");
            continue;
        }
        if (ip.b.length != ip.a.length || ip.a.length == 0 || ip.L.length < ip.L_len || ip.R.length < ip.L_len ||
            !ip.a.elements || !ip.b.elements || (ip.L_len && (!ip.L.elements || !ip.R.elements)))
            continue;   // stage_single's check: the single call returns false as well
        if (main.empty()) { abl = ip.a.length; Lr = ip.L_len; }
        (ip.a.length == abl && ip.L_len == Lr ? main : other).push_back(i);
    }
    if (!main.empty()) {   // the shape checks of the device batch (n a power of two, L_len <= log2 n)
        hipbp_proof_batch probe;
        memset(&probe, 0, sizeof probe);
        probe.count = 1; probe.n = n; probe.ab_len = abl; probe.L_len = Lr;
        const uint8_t dummy[1] = {0};
        probe.V = probe.A = probe.S = probe.T1 = probe.T2 = (const ge25519*)dummy;
        probe.t = probe.a = probe.b = probe.c = probe.x = (const fe25519*)dummy;
        probe.L = probe.R = (const ge25519*)dummy;
        int rc = check_batch(&probe, 1);
        if (rc != HIPBP_OK) return rc;
    }
    int dev0 = 0;   // the caller's current device: shard d runs on device (dev0 + d) % ndev, so
    BP_RET_ON(hipGetDevice(&dev0));   // num_gpus = 1 stays on it (one rank per GPU in a process group)
    const size_t M = main.size();
    std::vector<int> rcs(ng, HIPBP_OK);
    std::vector<std::string> errs(ng);
    std::vector<std::thread> workers;
    for (int d = 0; d < ng; d++) {
        const size_t lo = M * d / ng, hi = M * (d + 1) / ng;
        if (hi == lo) continue;
        workers.emplace_back([&, d, lo, hi]() {
            rcs[d] = host_shard((dev0 + d) % ndev, proofs, V, main.data() + lo, hi - lo, abl, Lr, n, G, H, h, ok);
            if (rcs[d] != HIPBP_OK) errs[d] = g_err;   // g_err is per thread
        });
    }
    for (auto& w : workers) w.join();
    for (int d = 0; d < ng; d++)
        if (rcs[d] != HIPBP_OK) {
            g_err = "device " + std::to_string(d) + ": " + errs[d];
            (void)hipSetDevice(dev0);
            return rcs[d];
        }
    BP_RET_ON(hipSetDevice(dev0));
    for (size_t i : other)
        ok[i] = verify_single(&proofs[i].ip_proof, &proofs[i], &V[i], nullptr, n, G, H, h) ? 1 : 0;
    return HIPBP_OK;
}

// ---- cuda_benchmark_* (declared at cuda_bulletproof.h:81-84, never defined by the reference)
static double now_s() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

void cuda_benchmark_multi_scalar_mul(int iterations, size_t vector_size) {
    std::vector<ge25519> pts(vector_size);
    std::vector<fe25519> sc(vector_size);
    for (size_t i = 0; i < vector_size; i++) {
        memset(&pts[i], 0, sizeof(ge25519));
        for (int k = 0; k < 4; k++) {
            pts[i].X.limbs[k] = 0x9E3779B97F4A7C15ull * (i + 1) ^ k;
            pts[i].Y.limbs[k] = 0xBF58476D1CE4E5B9ull * (i + 7) ^ k;
            sc[i].limbs[k] = 0x94D049BB133111EBull * (i + 3) + k;
        }
        pts[i].Z.limbs[0] = 1;
        sc[i].limbs[3] &= 0x7FFFFFFFFFFFFFFFull;
    }
    FieldVector s = {sc.data(), vector_size};
    PointVector p = {pts.data(), vector_size};
    ge25519 r;
    cuda_point_vector_multi_scalar_mul(&r, &s, &p);
    double t0 = now_s();
    for (int i = 0; i < iterations; i++) cuda_point_vector_multi_scalar_mul(&r, &s, &p);
    double dt = (now_s() - t0) / (iterations > 0 ? iterations : 1);
    printf("cuda_benchmark_multi_scalar_mul: n=%zu  %.3f ms/call  %.1f points/s\n", vector_size, dt * 1e3,
           vector_size / dt);
    fflush(stdout);
}

void cuda_benchmark_inner_product(int iterations, size_t vector_size) {
    std::vector<fe25519> a(vector_size), b(vector_size);
    for (size_t i = 0; i < vector_size; i++)
        for (int k = 0; k < 4; k++) {
            a[i].limbs[k] = 0x9E3779B97F4A7C15ull * (i + 1) + k;
            b[i].limbs[k] = 0xBF58476D1CE4E5B9ull * (i + 5) + k;
        }
    FieldVector av = {a.data(), vector_size}, bv = {b.data(), vector_size};
    fe25519 r;
    cuda_field_vector_inner_product(&r, &av, &bv);
    double t0 = now_s();
    for (int i = 0; i < iterations; i++) cuda_field_vector_inner_product(&r, &av, &bv);
    double dt = (now_s() - t0) / (iterations > 0 ? iterations : 1);
    printf("cuda_benchmark_inner_product: n=%zu  %.3f ms/call\n", vector_size, dt * 1e3);
    fflush(stdout);
}

void cuda_benchmark_field_operations(int iterations, size_t batch_size) {
    std::vector<fe25519> a(batch_size), b(batch_size), r(batch_size);
    for (size_t i = 0; i < batch_size; i++)
        for (int k = 0; k < 4; k++) {
            a[i].limbs[k] = 0x9E3779B97F4A7C15ull * (i + 1) + k;
            b[i].limbs[k] = 0xBF58476D1CE4E5B9ull * (i + 5) + k;
        }
    cuda_batch_field_mul(r.data(), a.data(), b.data(), batch_size);
    const char* names[3] = {"add", "mul", "square"};
    for (int op = 0; op < 3; op++) {
        double t0 = now_s();
        for (int i = 0; i < iterations; i++) {
            if (op == 0) cuda_batch_field_add(r.data(), a.data(), b.data(), batch_size);
            if (op == 1) cuda_batch_field_mul(r.data(), a.data(), b.data(), batch_size);
            if (op == 2) cuda_batch_field_square(r.data(), a.data(), batch_size);
        }
        double dt = (now_s() - t0) / (iterations > 0 ? iterations : 1);
        printf("cuda_benchmark_field_operations: %s x %zu  %.3f ms/call\n", names[op], batch_size, dt * 1e3);
        fflush(stdout);
    }
}

static uint64_t bench_mix(uint64_t x) {   // splitmix64: deterministic benchmark inputs
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

// max(iterations, 1) real bit_size-bit range proofs (values < 2^bit_size, random scalars shaped as
// generate_random_scalar, rp.cu:153-159) made by the GPU prover (hipbp_batch_generate_range_proof,
// same bits as generate_range_proof), then verified as the reference's host RangeProof structs:
// one cuda_range_proof_verify call per proof (the reference's per-proof entry point), and once
// more through hipbp_batch_range_proof_verify_host.  One line: per-call latency, batched rate,
// pass count, and whether the two verdict sets agree.
void cuda_benchmark_range_proof(int iterations, size_t bit_size) {
    const size_t n = bit_size;
    if (!is_pow2(n) || n > 64) {
        fprintf(stderr, "cuda_benchmark_range_proof: bit_size must be a power of two <= 64\n");
        return;
    }
    const size_t count = iterations > 0 ? std::min<size_t>((size_t)iterations, 65536) : 1;
    const size_t Lr = (size_t)log2i(n), ng = 2 * n + 2;
    uint64_t st = 0x5EEDull * 1000003 + n;
    auto rnd = [&]() { return bench_mix(st++); };
    // generators G[n] | H[n] | g | h: random X, Y < 2^255, Z = 1, T = X Y (the engine's fe25519_mul)
    std::vector<fe25519> X(ng), Y(ng), T(ng);
    for (size_t i = 0; i < ng; i++)
        for (int k = 0; k < 4; k++) {
            X[i].limbs[k] = rnd() & (k == 3 ? 0x7FFFFFFFFFFFFFFFull : ~0ull);
            Y[i].limbs[k] = rnd() & (k == 3 ? 0x7FFFFFFFFFFFFFFFull : ~0ull);
        }
    cuda_batch_field_mul(T.data(), X.data(), Y.data(), ng);
    std::vector<ge25519> gen(ng);
    for (size_t i = 0; i < ng; i++) {
        memset(&gen[i], 0, sizeof(ge25519));
        gen[i].X = X[i]; gen[i].Y = Y[i]; gen[i].Z.limbs[0] = 1; gen[i].T = T[i];
    }
    auto scalar = [&](fe25519& f) {   // generate_random_scalar's masks: byte 0 &= 0xF8, byte 31 &= 0x7F | 0x40
        for (int k = 0; k < 4; k++) f.limbs[k] = rnd();
        f.limbs[0] &= ~7ull;
        f.limbs[3] = (f.limbs[3] & 0x7FFFFFFFFFFFFFFFull) | 0x4000000000000000ull;
    };
    const size_t FE = sizeof(fe25519), GE = sizeof(ge25519);
    std::vector<fe25519> v(count), gamma(count), sL(count * n), sR(count * n), r4(count * 4);
    for (size_t p = 0; p < count; p++) {
        memset(&v[p], 0, FE);
        v[p].limbs[0] = n == 64 ? rnd() : rnd() & ((1ull << n) - 1);
        scalar(gamma[p]);
        for (size_t i = 0; i < n; i++) { scalar(sL[p * n + i]); scalar(sR[p * n + i]); }
        for (int i = 0; i < 4; i++) scalar(r4[p * 4 + i]);
    }
    Engine& e = engine_or_exit();
    const size_t Lc = Lr ? Lr : 1;
    // device: inputs | generators | outputs (V A S T1 T2 [count], taux mu t c x a b [count], L R [count Lr], valid)
    const size_t in_b = (count * (2 + 2 * n + 4)) * FE, gen_b = ng * GE;
    const size_t out_b = count * (5 * GE + 7 * FE + 2 * Lc * GE) + count;
    uint8_t* d = nullptr;
    BP_EXIT_ON(hipMalloc(&d, in_b + gen_b + out_b));
    fe25519* dv = (fe25519*)d;
    fe25519* dgam = dv + count;
    fe25519* dsL = dgam + count;
    fe25519* dsR = dsL + count * n;
    fe25519* dr4 = dsR + count * n;
    ge25519* dgen = (ge25519*)(d + in_b);
    uint8_t* o = d + in_b + gen_b;
    BP_EXIT_ON(hipMemcpy(dv, v.data(), count * FE, hipMemcpyHostToDevice));
    BP_EXIT_ON(hipMemcpy(dgam, gamma.data(), count * FE, hipMemcpyHostToDevice));
    BP_EXIT_ON(hipMemcpy(dsL, sL.data(), count * n * FE, hipMemcpyHostToDevice));
    BP_EXIT_ON(hipMemcpy(dsR, sR.data(), count * n * FE, hipMemcpyHostToDevice));
    BP_EXIT_ON(hipMemcpy(dr4, r4.data(), count * 4 * FE, hipMemcpyHostToDevice));
    BP_EXIT_ON(hipMemcpy(dgen, gen.data(), gen_b, hipMemcpyHostToDevice));
    hipbp_proof_out po;
    ge25519* og = (ge25519*)o;
    po.V = og; po.A = og + count; po.S = og + 2 * count; po.T1 = og + 3 * count; po.T2 = og + 4 * count;
    fe25519* of = (fe25519*)(og + 5 * count);
    po.taux = of; po.mu = of + count; po.t = of + 2 * count; po.c = of + 3 * count; po.x = of + 4 * count;
    po.a = of + 5 * count; po.b = of + 6 * count;
    ge25519* olr = (ge25519*)(of + 7 * count);
    po.L = olr; po.R = olr + count * Lc;
    po.valid = (uint8_t*)(olr + 2 * count * Lc);
    hipbp_prove_input pin{count, n, dv, dgam, dsL, dsR, dr4};
    if (hipbp_batch_generate_range_proof(&pin, dgen, dgen + n, dgen + 2 * n, dgen + 2 * n + 1, &po, nullptr) !=
        HIPBP_OK) {
        fprintf(stderr, "HIP error - %s\n", g_err.c_str());
        exit(EXIT_FAILURE);
    }
    BP_EXIT_ON(hipDeviceSynchronize());
    std::vector<uint8_t> host(out_b);
    BP_EXIT_ON(hipMemcpy(host.data(), o, out_b, hipMemcpyDeviceToHost));
    BP_EXIT_ON(hipFree(d));
    const ge25519* hg = (const ge25519*)host.data();
    const fe25519* hf = (const fe25519*)(hg + 5 * count);
    const ge25519* hlr = (const ge25519*)(hf + 7 * count);
    std::vector<fe25519> ha(hf + 5 * count, hf + 6 * count), hb(hf + 6 * count, hf + 7 * count);
    std::vector<ge25519> hL(hlr, hlr + count * Lc), hR(hlr + count * Lc, hlr + 2 * count * Lc);
    std::vector<RangeProof> proofs(count);
    std::vector<ge25519> V(hg, hg + count);
    for (size_t p = 0; p < count; p++) {
        RangeProof& rp = proofs[p];
        memset(&rp, 0, sizeof rp);
        rp.V = hg[p]; rp.A = hg[count + p]; rp.S = hg[2 * count + p]; rp.T1 = hg[3 * count + p];
        rp.T2 = hg[4 * count + p];
        rp.taux = hf[p]; rp.mu = hf[count + p]; rp.t = hf[2 * count + p];
        InnerProductProof& ip = rp.ip_proof;
        ip.n = n;
        ip.a.elements = &ha[p]; ip.a.length = 1;
        ip.b.elements = &hb[p]; ip.b.length = 1;
        ip.c = hf[3 * count + p];
        ip.x = hf[4 * count + p];
        ip.L.elements = Lr ? &hL[p * Lr] : nullptr; ip.L.length = Lr;
        ip.R.elements = Lr ? &hR[p * Lr] : nullptr; ip.R.length = Lr;
        ip.L_len = Lr;
    }
    PointVector Gv = {gen.data(), n}, Hv = {gen.data() + n, n};
    const ge25519 *g = &gen[2 * n], *h = &gen[2 * n + 1];
    std::vector<uint8_t> ok1(count), ok2(count);
    (void)cuda_range_proof_verify(&proofs[0], &V[0], n, &Gv, &Hv, g, h);   // warm-up (pipeline, tables)
    double t0 = now_s();
    for (size_t p = 0; p < count; p++) ok1[p] = cuda_range_proof_verify(&proofs[p], &V[p], n, &Gv, &Hv, g, h) ? 1 : 0;
    const double dt1 = now_s() - t0;
    if (hipbp_batch_range_proof_verify_host(proofs.data(), V.data(), count, n, &Gv, &Hv, g, h, 1, ok2.data()) !=
        HIPBP_OK) {
        fprintf(stderr, "HIP error - %s\n", g_err.c_str());
        exit(EXIT_FAILURE);
    }
    t0 = now_s();
    BP_EXIT_ON(hipbp_batch_range_proof_verify_host(proofs.data(), V.data(), count, n, &Gv, &Hv, g, h, 1, ok2.data())
                   == HIPBP_OK ? hipSuccess : hipErrorUnknown);
    const double dt2 = now_s() - t0;
    size_t pass = 0, agree = 0;
    for (size_t p = 0; p < count; p++) {
        pass += ok1[p];
        agree += ok1[p] == ok2[p];
    }
    printf("cuda_benchmark_range_proof: n=%zu  %zu proofs  cuda_range_proof_verify %.3f ms/call  "
           "batched (hipbp_batch_range_proof_verify_host) %.1f verifies/s  passes %zu/%zu  verdicts agree %zu/%zu\n",
           n, count, dt1 / count * 1e3, count / dt2, pass, count, agree, count);
    fflush(stdout);
}

}  // extern "C"
