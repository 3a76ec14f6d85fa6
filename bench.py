"""bench.py — batched 64-bit range-proof verification on MI355X (BASELINE.json metric).

  python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B] [--n 64]
  python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
      --master-port P bench.py --gpus N --steps K --warmup W

One step = cuda_range_proof_verify semantics (crv:82) over one batch of B = 1024 synthetic
64-bit proofs already resident in HBM (BASELINE configs[1]); every rank verifies its own
batches (weak scaling, no data-path collective: proofs are independent).  K steps are timed
between barrier + synchronize on both sides; the max over ranks is the step time.

Extra fields on the JSON line:
  roofline     the dominant kernel's algorithmic bytes / HIP-event launch time vs HBM peak
               (the path is VALU-integer bound), PMC traffic when profiled;
  cpu_baseline the CPU restatement (oracle/, test infrastructure) on a bounded sample, 1 thread;
  msm          2^20-point canonical-tree MSM points/s (BASELINE configs[2], per-point semantics);
               at N > 1 one MSM sharded over all ranks (cudabulletproof_amd/shard.py), strong scaling;
  ipa          4096-element inner-product-argument verifies/s (BASELINE configs[3]), rank 0;
  prove        generate_range_proof batched on the GPU, proofs/s, rank 0.
"""
import argparse
import hashlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: 8.0 TB/s spec
FE_B, GE_B = 32, 128


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--batch", type=int, default=1024, help="proofs per step per GPU")
    ap.add_argument("--n", type=int, default=64, help="range bits")
    ap.add_argument("--mode", choices=["pipeline", "oneshot"], default="pipeline",
                    help="pipeline: streaming verify pipeline, one tick (= one batch of work) per step; "
                         "oneshot: each step verifies one batch start to finish")
    ap.add_argument("--streams", type=int, default=2, help="oneshot mode: HIP streams batches rotate over")
    ap.add_argument("--pipes", type=int, default=2,
                    help="pipeline mode: verify pipelines on their own streams, batches alternate over them "
                         "(concurrent ticks fill each other's tails)")
    ap.add_argument("--msm-log2", type=int, default=20)
    ap.add_argument("--ipa-n", type=int, default=4096, help="configs[3]: inner-product-argument size")
    ap.add_argument("--ipa-batch", type=int, default=64, help="IPA proofs per pipeline tick")
    ap.add_argument("--ipa-steps", type=int, default=16)
    ap.add_argument("--no-ipa", action="store_true")
    ap.add_argument("--ipa-prefix-bits", type=int, default=14,
                    help="configs[3]: fixed-base prefix tables of G/H for fold round 0 (0 = none)")
    ap.add_argument("--prove-batch", type=int, default=65536, help="proofs per generate_range_proof batch")
    ap.add_argument("--prove-steps", type=int, default=4)
    ap.add_argument("--prove-streams", type=int, default=2, help="HIP streams prover batches rotate over")
    ap.add_argument("--no-prove", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--cpu-procs", type=int, default=16, help="processes for the parallel CPU baseline")
    ap.add_argument("--no-msm", action="store_true")
    ap.add_argument("--proofs", choices=["prover", "synthetic"], default="prover",
                    help="verify inputs: proofs made by the GPU prover from random 64-bit values (default) "
                         "or proof-shaped random data")
    ap.add_argument("--prefix-bits", type=int, default=22,
                    help="fixed-base prefix tables of the generators (hipbp_pipeline_prefix_tables; "
                         "0 = off): one-time setup, same bits")
    ap.add_argument("--shard-total", type=int, default=1 << 16, help="configs[4]: proofs in the sharded batch")
    ap.add_argument("--shard-batch", type=int, default=0,
                    help="configs[4]: proofs per pipeline push (0: auto from the rank's shard size)")
    ap.add_argument("--no-shard", action="store_true")
    ap.add_argument("--host-count", type=int, default=32768, help="proofs per host-struct API call")
    ap.add_argument("--no-host", action="store_true")
    ap.add_argument("--rehearse", action="store_true",
                    help="exercise the N>1 path on one GPU (all ranks on cuda:0, gloo collectives); not a measurement")
    return ap.parse_args()


TASK_B = GE_B + FE_B + GE_B   # one scalar-mult task: point + scalar in, term out


def alg_bytes(kernel, B, n, ab_len):
    """Algorithmic HBM bytes of all launches of `kernel` for one batch (inputs read + outputs written)."""
    if kernel == "k_terms":   # every scalar multiplication of a verify: 2 MSMs, all fold rounds, t*h, c*Q, a0*G', b0*H'
        return B * sm_per_verify(n) * TASK_B
    return None


def sm_per_verify(n):
    Lr = n.bit_length() - 1
    return 2 * n + sum(4 * (n >> (r + 1)) for r in range(Lr)) + 4


def proof_bytes(n, ab_len):
    Lr = n.bit_length() - 1
    return 5 * GE_B + 3 * FE_B + 2 * ab_len * FE_B + 2 * Lr * GE_B   # V,A,S,T1,T2, t,c,x, a,b, L,R


def _cpu_sample(n, count):
    from cudabulletproof_amd import synth
    s = synth.proofs(count, n, seed=777)
    heads = [np.concatenate([s[k][p] for k in ("V", "A", "S", "T1", "T2")] +
                            [np.zeros(8, np.uint64), s["t"][p], s["c"][p], s["x"][p]]) for p in range(count)]
    return s, heads


def _cpu_worker(args):
    """One process of the parallel CPU baseline: verify proofs [lo, hi) with the reference build."""
    n, lo, hi, seconds = args
    from oracle import pyoracle
    R = pyoracle.Reference()
    G, H = R.base_points(n, 1), R.base_points(n, 2)
    g, h = R.gh()
    s, heads = _cpu_sample(n, hi)
    done, t0 = 0, time.perf_counter()
    for p in range(lo, hi):
        R.cuda_range_proof_verify(dict(head=heads[p], V=s["V"][p], a=s["a"][p], b=s["b"][p], L=s["L"][p],
                                       R=s["R"][p]), n, G, H, g, h)
        done += 1
        if time.perf_counter() - t0 > seconds:
            break
    return done, time.perf_counter() - t0


def cpu_baseline(n, seconds, procs):
    """The reference's own cuda_range_proof_verify (its host sources compiled by oracle/build_ref.sh
    into oracle/_ref/libbpref.so, the two MSMs host-emulated with the canonical tree) on this host:
    1 thread on a bounded sample (`value`), and `procs` processes side by side (`parallel`).
    Falls back to the CPU restatement (oracle/bp_oracle.c, kind "port") if the build is absent."""
    from oracle import pyoracle
    if not pyoracle.have_reference():
        O = pyoracle.Oracle()
        G, H = O.base_points(n, 1), O.base_points(n, 2)
        g, h = O.gh()
        s, heads = _cpu_sample(n, 64)
        done, t0 = 0, time.perf_counter()
        for p in range(64):
            O.cuda_range_proof_verify(heads[p], s["V"][p], n, s["a"][p], s["b"][p], s["L"][p], s["R"][p], G, H, g, h)
            done += 1
            if time.perf_counter() - t0 > seconds:
                break
        dt = time.perf_counter() - t0
        return {"value": done / dt, "unit": "verifies/s", "cores": 1, "kind": "port",
                "sample": f"{done} synthetic {n}-bit proofs, oracle/bp_oracle.c, 1 thread, {dt:.1f} s",
                "cpu": cpu_model()}
    done, dt = _cpu_worker((n, 0, 512, seconds))
    out = {"value": done / dt, "unit": "verifies/s", "cores": 1, "kind": "reference",
           "sample": f"{done} synthetic {n}-bit proofs, the reference's cuda_range_proof_verify (oracle/_ref), "
                     f"1 thread, {dt:.1f} s", "cpu": cpu_model()}
    if procs > 1:
        import multiprocessing as mp
        per = 16
        with mp.get_context("spawn").Pool(procs) as pool:
            t0 = time.perf_counter()
            res = pool.map(_cpu_worker, [(n, k * per, (k + 1) * per, seconds) for k in range(procs)])
            wall = time.perf_counter() - t0
        tot = sum(r[0] for r in res)
        out["parallel"] = {"value": sum(r[0] / r[1] for r in res), "unit": "verifies/s", "cores": procs,
                           "sample": f"{tot} proofs over {procs} processes ({per} each), {wall:.1f} s wall"}
    return out


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def pmc(kernel, key, config=None):
    """A per-launch PMC figure for `kernel` from the committed rocprofv3 summary, if present and
    (when `config` is given) collected on the same bench configuration."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        d = json.load(open(path))
        if config is not None and d.get("config") != config:
            return None
        return d.get(kernel, {}).get(key)
    except (OSError, ValueError):
        return None


# VALU issue peak (the binding resource of this path): 1024 SIMDs x 2.4 GHz / 4 cycles per
# wave64 instruction.  A SIMD-32 issues a wave64 instruction in 2 passes; the integer
# instructions the limb arithmetic is made of (v_mad_u64_u32, v_addc/v_add_co, v_cmp,
# v_cndmask, v_lshl_add_u64, v_alignbit) take 4 cycles per wave-instruction (tools/ubench_enc.hip
# measures 4.3-5.1 at the nominal clock); only plain 32-bit add/sub/logic/mov take 2.
VALU_PEAK_WINSTR = 1024 * 2.4e9 / 4


def msm_leg(args, dev, world, rank, T):
    """2^k-point canonical-tree MSM; each rank holds its shard (shard.msm_shard_bounds) and the
    roots meet in one all_gather + tree (bit-exact with one GPU).  Timed between barriers,
    max over ranks."""
    import torch
    import torch.distributed as dist
    from cudabulletproof_amd import shard, synth
    nm = 1 << args.msm_log2
    lo, hi = shard.msm_shard_bounds(nm, world, rank)
    sc, pts = synth.msm_config3(lo, hi, dev)   # SURVEY §8(d) config 3 inputs, this rank's rows
    scd, ptd = T(sc), T(pts)
    del sc, pts
    shard.sharded_msm(scd, ptd, nm)
    torch.cuda.synchronize(dev)
    reps = 3
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t1 = time.perf_counter()
    for _ in range(reps):
        res = shard.sharded_msm(scd, ptd, nm)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    mdt = (time.perf_counter() - t1) / reps
    if world > 1:
        t = torch.tensor([mdt], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        mdt = float(t.item())
    digest = hashlib.sha256(res.cpu().numpy().tobytes()).hexdigest()[:16]
    golden_ok = None   # tests/golden/msm_2p20.json: the CPU restatement's result for the 2^20 inputs
    gpath = os.path.join(os.path.dirname(os.path.abspath(__file__)), "tests", "golden", "msm_2p20.json")
    gold = None
    if os.path.exists(gpath):
        with open(gpath) as f:
            gold = json.load(f)
        if gold["n"] == nm:
            golden_ok = digest == gold["digest"]
        else:
            gold = None
    pip = None
    if world == 1:   # the labelled alternative: Pippenger window 12 on the same inputs, one GPU
        import cudabulletproof_amd as bp
        out = torch.zeros(16, dtype=torch.int64, device=dev)
        bp.msm_pippenger(out, scd, ptd, 12)
        torch.cuda.synchronize(dev)
        t1 = time.perf_counter()
        for _ in range(reps):
            bp.msm_pippenger(out, scd, ptd, 12)
        torch.cuda.synchronize(dev)
        pdt = (time.perf_counter() - t1) / reps
        pd = hashlib.sha256(out.cpu().numpy().tobytes()).hexdigest()[:16]
        # throughput: independent MSMs alternate over two streams (per-stream workspaces), so one
        # MSM's latency-bound chains (chunks, Horner) run beside the other's sort and bucket trees
        ns, m = 2, 4 * reps
        sts = [torch.cuda.Stream(dev) for _ in range(ns)]
        outs = torch.zeros(m, 16, dtype=torch.int64, device=dev)
        torch.cuda.synchronize(dev)   # the zero fill is on torch's stream, the MSMs are not
        for i in range(ns):
            bp.msm_pippenger(outs[i], scd, ptd, 12, stream=sts[i])
        torch.cuda.synchronize(dev)
        t1 = time.perf_counter()
        for k in range(m):
            bp.msm_pippenger(outs[k], scd, ptd, 12, stream=sts[k % ns])
        torch.cuda.synchronize(dev)
        tdt = (time.perf_counter() - t1) / m
        same = bool((outs == out.unsqueeze(0)).all().item())
        # batched: hipbp_msm_pippenger_batch, bc MSMs over the same points in one sort/tree pass
        # (MSM j's scalars = the config-3 scalars rolled by j rows), bc-batches on two streams
        bc = 4
        sb = torch.cat([torch.roll(scd, j, 0) for j in range(bc)]).contiguous()
        want = torch.zeros(bc, 16, dtype=torch.int64, device=dev)
        for j in range(bc):
            bp.msm_pippenger(want[j], sb[j * nm:(j + 1) * nm], ptd, 12)
        bouts = [torch.zeros(bc, 16, dtype=torch.int64, device=dev) for _ in range(ns)]
        torch.cuda.synchronize(dev)
        for i in range(ns):
            bp.msm_pippenger_batch(bouts[i], sb, ptd, 12, stream=sts[i])
        torch.cuda.synchronize(dev)
        bm = 2 * reps
        t1 = time.perf_counter()
        for k in range(bm):
            bp.msm_pippenger_batch(bouts[k % ns], sb, ptd, 12, stream=sts[k % ns])
        torch.cuda.synchronize(dev)
        bdt = (time.perf_counter() - t1) / (bm * bc)
        bsame = all(bool((o == want).all().item()) for o in bouts)
        del sb
        pip = {"metric": "MSM points/sec (Pippenger, window 12)", "value": nm / tdt, "unit": "points/s",
               "ms_per_msm": tdt * 1e3, "msms_in_flight": ns, "msms_timed": m, "all_results_equal": same,
               "single_stream": {"value": nm / pdt, "ms_per_msm": pdt * 1e3},
               "batched": {"value": nm / bdt, "ms_per_msm": bdt * 1e3, "msms_per_call": bc, "streams": ns,
                           "msms_timed": bm * bc, "all_match_single_calls": bsame,
                           "api": "hipbp_msm_pippenger_batch (same points, count scalar sets)"},
               "window_bits": 12, "result_sha256": pd,
               "matches_oracle_golden": (pd == gold["pippenger_w12"]["digest"]) if gold else None,
               "semantics": "labelled alternative (hipbp_msm_pippenger): bucket algorithm over the reference's "
                            "arithmetic, bit-exact with oracle/ orc_msm_pippenger, NOT the reference's MSM bits "
                            "(non-associative arithmetic; the graded MSM is the canonical-tree leg above)"}
    psh = None
    if world > 1:   # Pippenger over N GPUs: window ranges per rank, one all_gather of window sums, Horner
        import cudabulletproof_amd as bp
        if lo != 0 or hi != nm:
            del scd, ptd
            sc, pts = synth.msm_config3(0, nm, dev)   # every rank holds all points (windows split, not points)
            scd, ptd = T(sc), T(pts)
            del sc, pts
        res = shard.sharded_msm_pippenger(scd, ptd, 12)
        torch.cuda.synchronize(dev)
        dist.barrier()
        torch.cuda.synchronize(dev)
        t1 = time.perf_counter()
        for _ in range(reps):
            res = shard.sharded_msm_pippenger(scd, ptd, 12)
        torch.cuda.synchronize(dev)
        dist.barrier()
        sdt = (time.perf_counter() - t1) / reps
        t = torch.tensor([sdt], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        sdt = float(t.item())
        sd = hashlib.sha256(res.cpu().numpy().tobytes()).hexdigest()[:16]
        w0, w1 = shard.pippenger_window_bounds(12, world, rank)
        psh = {"metric": "MSM points/sec (Pippenger, window 12, windows sharded over the ranks)", "value": nm / sdt,
               "unit": "points/s", "ms_per_msm": sdt * 1e3, "n_gpus": world, "scaling": "strong",
               "windows_rank0": [w0, w1], "result_sha256": sd,
               "matches_oracle_golden": (sd == gold["pippenger_w12"]["digest"]) if gold else None,
               "collective": "one all_gather of the largest window range x 128 B per rank (RCCL), then the Horner "
                             "chain on every rank (shard.sharded_msm_pippenger)"}
    return {"metric": "MSM points/sec", "value": nm / mdt, "unit": "points/s", "points": nm,
            "ms_per_msm": mdt * 1e3, "n_gpus": world, "scaling": "strong" if world > 1 else None,
            "semantics": "canonical-tree per-point double-and-add (SURVEY A9); shards + all_gather + tree at N>1",
            "result_sha256": digest, "matches_oracle_golden": golden_ok, "pippenger": pip,
            "pippenger_sharded": psh}


def ipa_leg(args, dev):
    """configs[3]: cuda_inner_product_verify semantics at n = 4096 on
    batches of synthetic IPA proofs streamed through the pipeline in inner-product mode, each
    proof's P = the canonical-tree MSM of its a||b over G||H (8192 points, hipbp_msm_batch on the
    pipeline's stream, inside the timed region); also timed with P given."""
    import torch
    import cudabulletproof_amd as bp
    from cudabulletproof_amd import synth
    n, B = args.ipa_n, args.ipa_batch
    G, H, _, h = synth.generators(n, dev)
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a).view(np.int64)).to(dev)
    Gd, Hd, Qd = T(G), T(H), T(h)
    GH = torch.cat([Gd, Hd]).contiguous()
    npipe = max(1, args.pipes)   # as the verify leg: concurrent pipelines on their own streams
    nb = 2 * npipe
    batches = [bp.RangeProofBatch.from_numpy(n, synth.proofs(B, n, seed=90 + i), dev) for i in range(nb)]
    wit = [T(synth._rand_fe(np.random.default_rng(60 + i), (B * 2 * n,))) for i in range(nb)]   # a||b per proof
    Ps = [torch.zeros(B, 16, dtype=torch.int64, device=dev) for _ in range(nb)]
    oks = [torch.zeros(B, dtype=torch.uint8, device=dev) for _ in range(nb)]
    streams = [torch.cuda.Stream(dev) for _ in range(npipe)]
    pipes = [bp.VerifyPipeline(B, n, Gd, Hd, Qd, range_mode=False, stream=st) for st in streams]
    pipe = pipes[0]
    gens = None
    if args.ipa_prefix_bits > 0:   # one table set shared by both pipelines (fold round 0 is on G, H)
        t0 = time.perf_counter()
        gens = bp.Generators(n, Gd, Hd, Qd, Qd, prefix_bits=args.ipa_prefix_bits)
        for pp in pipes:
            pp.use_gens(gens)
        torch.cuda.synchronize(dev)
        tables = {"bits": args.ipa_prefix_bits, "GB": gens.nbytes_tables() / 1e9,
                  "build_s": time.perf_counter() - t0}

    P_same = None
    if gens is not None:   # the tables change no bits: P of batch 0 both ways, outside the timed region
        pa, pb = torch.zeros_like(Ps[0]), torch.zeros_like(Ps[0])
        bp.msm_batch(pa, wit[0], GH)
        bp.msm_batch_gens(pb, wit[0], gens)
        torch.cuda.synchronize(dev)
        P_same = bool(torch.equal(pa, pb))

    def tick(k, with_P):   # P of batch k on its pipeline's stream (per-stream MSM workspaces), then the tick
        j = k % npipe
        if with_P:   # over the generator set's G||H with its prefix tables when there is one (same bits)
            if gens is not None:
                bp.msm_batch_gens(Ps[k % nb], wit[k % nb], gens, stream=streams[j])
            else:
                bp.msm_batch(Ps[k % nb], wit[k % nb], GH, stream=streams[j])
        pipes[j].push(batches[k % nb], oks[k % nb], P_in=Ps[k % nb])

    res = {}
    steps = max(args.ipa_steps, npipe) // npipe * npipe
    for with_P in (True, False):
        for k in range((pipe.depth - 1) * npipe):   # fill: every timed tick then completes one batch
            tick(k, with_P)
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for k in range(steps):
            tick(k, with_P)
        torch.cuda.synchronize(dev)
        res[with_P] = time.perf_counter() - t0
        for pp in pipes:
            pp.flush()
        torch.cuda.synchronize(dev)
    for pp in pipes:
        pp.close()
    if gens is not None:
        gens.close()
    sm = 4 * (n - 1) + 3   # fold rounds + a0*G', b0*H', c*Q (crv:160-296)
    dt = res[True]
    return {"metric": f"{n}-element inner-product-argument verifies/sec", "value": B * steps / dt,
            "unit": "verifies/s", "batch": B, "n": n, "ms_per_tick": dt / steps * 1e3, "pipelines": npipe,
            "scalar_mults_per_verify": sm + 2 * n, "scalar_mults_per_s": B * steps * (sm + 2 * n) / dt,
            "value_P_given": B * steps / res[False],
            "semantics": "P = canonical-tree MSM(a||b, G||H) (hipbp_msm_batch_gens) + cuda_inner_product_verify "
                         "(crv:130)", "pipeline_depth": pipe.depth,
            "prefix_tables": tables if gens is not None else None, "P_tables_equal_plain": P_same}


def shard_push_batch(args, shard_size, npipe):
    """Proofs per push for a rank's shard.  A pushed batch completes depth - 1 ticks after its push,
    and the drain ticks (fold rounds 3..5, final terms of the last batches) are latency-bound, so a
    small shard (8192 proofs per rank at N = 8) goes through in fewer, larger pushes: ≈2 per
    pipeline, at most 4096 proofs each; a large one keeps the bench's B (measured)."""
    if args.shard_batch > 0:
        return args.shard_batch
    per = -(-shard_size // (2 * npipe))
    Bs = args.batch
    while Bs < per and Bs < 4096:
        Bs *= 2
    return Bs


def shard_leg(args, dev, world, rank, pipes, gens, G, H, g, h, streams=None):
    """configs[4]: ONE batch of 2^16 64-bit proofs (1024 x 4 distinct proofs, tiled: the kernels do
    not dedupe) split into equal contiguous shards over the ranks (shard.shard_bounds).  Each rank
    verifies its shard through its pipelines; the pass counts meet in one all_reduce(SUM) and the
    2^16 verdict bytes in one all_gather over RCCL (every rank ends with all verdicts).  Timed
    from a barrier to the end of the collectives (pipeline fill and drain included), max over ranks;
    strong scaling: the same 2^16 proofs whatever N."""
    import torch
    import torch.distributed as dist
    import cudabulletproof_amd as bp
    from cudabulletproof_amd import shard, synth
    B, n, total = args.batch, args.n, args.shard_total
    lo, hi = shard.shard_bounds(total, world, rank)
    tiles = []
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a).view(np.int64)).to(dev)
    for t in range(4):   # rank-independent tiles: the global set is the same for every N
        pi = {k: T(v) for k, v in synth.prove_inputs(B, n, seed=5001 + t).items()}
        out = bp.batch_generate_range_proof(n, pi["v"], pi["gamma"], pi["sL"], pi["sR"], pi["rnd"], G, H, g, h,
                                            gens=gens)
        tiles.append({k: out[k] for k in bp.RangeProofBatch.FIELDS})
    torch.cuda.synchronize(dev)
    Bs = shard_push_batch(args, hi - lo, len(pipes))
    own = []
    if Bs != B:   # pipelines sized for the larger pushes, on the same streams
        own = [bp.VerifyPipeline(Bs, n, G, H, h, stream=streams[i] if streams else None)
               for i in range(len(pipes))]
        if gens is not None:
            for pp in own:
                pp.use_gens(gens)
        pipes = own
    def rows(j0, m):   # proofs [j0, j0 + m) of the global set: proof j is tile (j // B) % 4, row j % B
        parts, j = [], j0
        while j < j0 + m:
            k = min(B - j % B, j0 + m - j)
            parts.append(((j // B) % 4, j % B, k))
            j += k
        return {f: torch.cat([tiles[t][f][r0:r0 + k] for t, r0, k in parts]) for f in bp.RangeProofBatch.FIELDS}
    jobs, j = [], lo
    while j < hi:
        m = min(Bs, hi - j)
        jobs.append((j, m))
        j += m
    batches = [bp.RangeProofBatch(n, **rows(j0, m)) for j0, m in jobs]
    ok = torch.zeros(hi - lo, dtype=torch.uint8, device=dev)
    offs = np.cumsum([0] + [m for _, m in jobs])
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for k, b in enumerate(batches):
        pipes[k % len(pipes)].push(b, ok[offs[k]:offs[k + 1]])
    for pp in pipes:
        pp.flush()
    torch.cuda.synchronize(dev)   # the pipelines' streams have written every verdict
    passes = ok.sum(dtype=torch.int64)
    allv = ok
    if world > 1:
        dist.all_reduce(passes, op=dist.ReduceOp.SUM)
        nccl = dist.get_backend() == "nccl"   # --rehearse runs gloo, which gathers host tensors
        allv = shard.gather_verdicts(ok if nccl else ok.cpu(), total)
    torch.cuda.synchronize(dev)
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    import hashlib as _h
    for pp in own:
        pp.close()
    return {"metric": "2^16-proof 64-bit range-proof batch verify (BASELINE configs[4])", "value": total / dt,
            "push_batch": Bs,
            "unit": "verifies/s", "proofs": total, "n_gpus": world, "scaling": "strong", "ms": dt * 1e3,
            "passes": int(passes.item()), "verdicts_sha256": _h.sha256(allv.cpu().numpy().tobytes()).hexdigest()[:16],
            "collectives": "all_reduce(SUM) of pass counts + all_gather of the verdict bytes (RCCL at N > 1)",
            "data": "1024 x 4 distinct GPU-prover proofs (rank-independent seeds), tiled to 2^16"}


def host_leg(args, batches, G, H, g, h):
    """The host-struct entry point hipbp_batch_range_proof_verify_host: an array of the reference's
    own RangeProof structs in host memory (cuda_range_proof_verify semantics per proof), so the
    rate includes packing, one H2D, the pipeline and one D2H (PCIe-inclusive; never `value`)."""
    import ctypes
    import cudabulletproof_amd as bp
    host = [{k: getattr(b, k).cpu().numpy().view(np.uint64) for k in bp.RangeProofBatch.FIELDS} for b in batches]
    count = args.host_count
    keep, proofs, V = [], [], []
    for i in range(count):
        a = host[(i // len(host[0]["V"])) % len(host)]
        j = i % len(a["V"])
        head = np.concatenate([a[k][j] for k in ("V", "A", "S", "T1", "T2")] +
                              [np.zeros(8, np.uint64), a["t"][j], a["c"][j], a["x"][j]])
        proofs.append(bp._range_proof_struct(dict(head=head, a=a["a"][j], b=a["b"][j], L=a["L"][j], R=a["R"][j]),
                                             args.n, keep))
        V.append(a["V"][j])
    arr = (bp.RangeProofC * count)(*proofs)
    V = np.ascontiguousarray(np.stack(V))
    G, H, g, h = (np.ascontiguousarray(x.cpu().numpy().view(np.uint64)) for x in (G, H, g, h))
    gv, hv = bp.PointVector(G.ctypes.data, len(G)), bp.PointVector(H.ctypes.data, len(H))
    ok = np.zeros(count, np.uint8)
    L = bp.lib()
    call = lambda: bp._chk(L.hipbp_batch_range_proof_verify_host(
        arr, ctypes.c_void_p(V.ctypes.data), ctypes.c_size_t(count), ctypes.c_size_t(args.n), ctypes.byref(gv),
        ctypes.byref(hv), ctypes.c_void_p(g.ctypes.data), ctypes.c_void_p(h.ctypes.data), ctypes.c_int(1),
        ctypes.c_void_p(ok.ctypes.data)))
    call()
    reps = 2
    t1 = time.perf_counter()
    for _ in range(reps):
        call()
    dt = (time.perf_counter() - t1) / reps
    return {"metric": "64-bit range-proof verifies/sec, host RangeProof structs (PCIe-inclusive)",
            "value": count / dt, "unit": "verifies/s", "proofs": count, "ms": dt * 1e3, "passes": int(ok.sum()),
            "n_gpus": 1, "entry_point": "hipbp_batch_range_proof_verify_host",
            "bytes_h2d": int(count * (5 * 128 + 3 * 32 + 2 * 32 + 2 * 128 * int(np.log2(args.n))))}


def prove_leg(args, dev, gens=None):
    """§8(f) rank 1: generate_range_proof (rp.cu:1159) batched on the GPU, n = args.n, synthetic
    values and random scalars; proofs/s over whole batches (inputs resident in HBM)."""
    import torch
    import cudabulletproof_amd as bp
    from cudabulletproof_amd import synth
    n, B = args.n, args.prove_batch
    G, H, g, h = synth.generators(n, dev)
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a).view(np.int64)).to(dev)
    Gd, Hd, gd, hd = T(G), T(H), T(g), T(h)
    pi = {k: T(v) for k, v in synth.prove_inputs(B, n).items()}
    # two streams: one batch's latency-bound stages (T terms, IPA rounds, chains) run under the
    # other batch's term launches (each stream has its own prover workspace in the engine)
    # (different priorities: HIP maps streams onto at most GPU_MAX_HW_QUEUES hardware queues and two
    # same-priority streams created after the verify legs' streams can share one, which serializes them)
    lo, hi = torch.cuda.Stream.priority_range()
    ns = max(1, args.prove_streams)
    streams = [torch.cuda.Stream(dev, priority=max(hi, lo - k)) for k in range(ns)]
    torch.cuda.synchronize(dev)
    run = lambda k: bp.batch_generate_range_proof(n, pi["v"], pi["gamma"], pi["sL"], pi["sR"], pi["rnd"], Gd, Hd,
                                                  gd, hd, stream=streams[k % ns], gens=gens)
    outs = [run(k) for k in range(ns)]
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for k in range(args.prove_steps):
        outs[k % ns] = run(k)
    torch.cuda.synchronize(dev)
    dt = (time.perf_counter() - t0) / args.prove_steps
    same = all(torch.equal(outs[0][k], outs[-1][k]) for k in ("A", "S", "T1", "L", "R"))
    return {"metric": f"{n}-bit range proofs generated/sec", "value": B / dt, "unit": "proofs/s", "batch": B,
            "streams": ns, "ms_per_batch": dt * 1e3, "valid": int(outs[0]["valid"].sum().item()),
            "deterministic_across_streams": same,
            "semantics": "generate_range_proof + inner_product_prove + fix_inner_product_proof (rp.cu:1159)",
            "prefix_bits": gens.bits if gens is not None else 0}


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    import cudabulletproof_amd as bp
    from cudabulletproof_amd import synth

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # CPU baseline first, before this process touches the GPU: its worker processes are started
    # from a process with no HIP state (no fork/exec of a GPU-initialised process)
    cpu = None
    if not args.no_cpu and rank == 0 and world == 1:
        cpu = cpu_baseline(args.n, args.cpu_seconds, args.cpu_procs)
    if args.rehearse:   # N>1 code path on a 1-GPU box: every rank on cuda:0, gloo instead of RCCL
        local = 0
        args.prefix_bits = min(args.prefix_bits, 16)   # every rank's tables share the one GPU
    if world > 1:
        torch.cuda.set_device(local)
        if args.rehearse:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    bp.lib()
    bp.require_gpu()

    B, n = args.batch, args.n
    G, H, g, h = synth.generators(n, dev)
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a).view(np.int64)).to(dev)
    Gd, Hd, gd, hd = T(G), T(H), T(g), T(h)
    # one generator set (snapshot + fixed-base prefix tables): the input prover, the verify pipeline
    # and the prover leg share it; one-time setup per generator set, outside every timed region
    prefix = None
    gens = None
    if args.prefix_bits:
        torch.cuda.synchronize(dev)
        tp = time.perf_counter()
        gens = bp.Generators(n, Gd, Hd, gd, hd, prefix_bits=args.prefix_bits)
        prefix = {"bits": args.prefix_bits, "bases": 2 * n + 2, "GB": gens.nbytes_tables() / 1e9,
                  "build_s": time.perf_counter() - tp}
    nb = 4
    if args.proofs == "prover":   # real 64-bit range proofs from the GPU prover (bit-exact with the reference's)
        batches = []
        for i in range(nb):
            pi = {k: T(v) for k, v in synth.prove_inputs(B, n, seed=1 + 1000 * rank + i).items()}
            out = bp.batch_generate_range_proof(n, pi["v"], pi["gamma"], pi["sL"], pi["sR"], pi["rnd"], Gd, Hd, gd, hd,
                                                gens=gens)
            torch.cuda.synchronize(dev)
            batches.append(bp.RangeProofBatch(n, **{k: out[k] for k in bp.RangeProofBatch.FIELDS}))
    else:
        batches = [bp.RangeProofBatch.from_numpy(n, synth.proofs(B, n, seed=1 + 1000 * rank + i), dev)
                   for i in range(nb)]
    # configs[2] first, before the verify streams exist: hipbp_msm_pippenger overlaps its chains on
    # an internal side stream, which needs a hardware queue of its own (HIP spreads streams over
    # GPU_MAX_HW_QUEUES = 4; with the verify pipelines' streams bound first it shared one: 312 -> 190
    # M points/s); at N > 1 one MSM sharded over all ranks (strong scaling)
    msm = None
    if not args.no_msm:
        msm = msm_leg(args, dev, world, rank, T)
    ns = max(1, args.streams, args.pipes)
    streams = [torch.cuda.Stream(dev) for _ in range(ns)]
    oks = [torch.zeros(B, dtype=torch.uint8, device=dev) for _ in range(max(ns, nb))]
    stream = torch.cuda.current_stream(dev)
    torch.cuda.synchronize(dev)
    pipe = None
    pipes = []
    if args.mode == "pipeline":
        npipe = max(1, args.pipes)
        pipes = [bp.VerifyPipeline(B, n, Gd, Hd, hd, stream=streams[i]) for i in range(npipe)]
        for pp in pipes:
            if gens is not None:
                pp.use_gens(gens)
        pipe = pipes[0]

        def step(k):   # one tick: stage s of the batch pushed s ticks earlier, for every s
            pipes[k % npipe].push(batches[k % nb], oks[k % nb])
        warm = max(args.warmup, pipe.depth * npipe)   # fill the pipelines before timing
    else:
        def step(k):
            bp.batch_range_proof_verify(batches[k % nb], Gd, Hd, gd, hd, oks[k % ns], stream=streams[k % ns])
        warm = max(args.warmup, 1)

    for k in range(warm):
        step(k)
    for pp in pipes:
        pp.flush()
    torch.cuda.synchronize(dev)
    passes_warm = int(oks[0].sum().item())

    if pipe:   # refill (flush drained it) so every timed tick carries a full batch of work
        for k in range((pipe.depth - 1) * len(pipes)):
            step(k)
        torch.cuda.synchronize(dev)
    bp.timing_enable(True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for k in range(args.steps):
        step(k)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    stats = bp.timing_collect()
    bp.timing_enable(False)
    for pp in pipes:
        pp.flush()
    torch.cuda.synchronize(dev)
    sharded = None
    if pipes and not args.no_shard:   # configs[4] on the same pipelines (all ranks take part)
        sharded = shard_leg(args, dev, world, rank, pipes, gens, Gd, Hd, gd, hd, streams)
    for pp in pipes:
        pp.close()
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
        c = torch.tensor([passes_warm], dtype=torch.int64, device=dev)
        dist.all_reduce(c, op=dist.ReduceOp.SUM)
        passes_warm = int(c.item())

    total = B * args.steps * world
    value = total / dt

    # dominant kernel + live roofline (HIP events on the verify stream)
    kern_ms = {k: v[0] for k, v in stats.items() if v[1]}
    dom = max(kern_ms, key=kern_ms.get)
    launches = stats[dom][1]
    avg_ms = stats[dom][0] / launches
    ab_batch = alg_bytes(dom, B, n, 1)
    per_launch = ab_batch * args.steps / launches if ab_batch else None
    achieved = (per_launch / (avg_ms * 1e-3)) / 1e9 if per_launch else None
    pcfg = {"batch_per_gpu": B, "n": n, "prefix_bits": prefix["bits"] if prefix else 0}
    # with P > 1 pipelines two ticks run concurrently, so a launch's own duration includes its
    # overlap with the other's: the aggregate rate (work of every launch in the timed region / the
    # region's wall time) is reported beside the per-launch one
    agg = ab_batch * args.steps / dt / 1e9 if ab_batch else None
    roofline = {
        "bound": "hbm", "kernel": dom, "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
        "frac": (achieved / HBM_PEAK_GBS) if achieved else None, "traffic": pmc(dom, "bytes_per_launch", pcfg),
        "achieved_aggregate": agg, "frac_aggregate": agg / HBM_PEAK_GBS if agg else None,
        "avg_launch_ms": avg_ms, "launches": launches, "concurrent_pipelines": len(pipes) or None,
        "kernel_ms_share": {k: round(v / sum(kern_ms.values()), 4) for k, v in kern_ms.items()},
        "binding": "VALU integer (not HBM, not MFMA): see DESIGN.md and valu_roofline",
        "scalar_mults_per_s": value * sm_per_verify(n),
    }
    vi = pmc(dom, "valu_instr_per_launch", pcfg)
    vagg = vi * launches / dt if vi else None   # all launches of the timed region / its wall time
    valu_roofline = {
        "kernel": dom, "unit": "wave64 VALU instr/s", "peak": VALU_PEAK_WINSTR,
        "instr_per_launch": vi, "achieved": vagg, "frac": vagg / VALU_PEAK_WINSTR if vagg else None,
        "achieved_per_launch": vi / (avg_ms * 1e-3) if vi else None,
        "valu_busy_pct": pmc(dom, "valu_busy_pct", pcfg), "pmc_config": pcfg,
        "source": "SQ_INSTS_VALU per steady-state launch (profiles/pmc_traffic.json) x launches in the timed "
                  "region / its wall time (per_launch: / the live HIP-event launch time, which overlaps "
                  "the other pipeline's launch when pipes > 1)",
    }


    ipa = None
    if not args.no_ipa and rank == 0:   # configs[3]: single-GPU
        ipa = ipa_leg(args, dev)
        ipa["n_gpus"] = 1

    host_api = None
    if not args.no_host and rank == 0 and world == 1:
        host_api = host_leg(args, batches, Gd, Hd, gd, hd)

    prove = None
    if not args.no_prove and rank == 0:
        prove = prove_leg(args, dev, gens)
        prove["n_gpus"] = 1


    if rank == 0:
        line = {
            "metric": "64-bit range-proof verifies/sec (batched)", "value": value, "unit": "verifies/s",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup, "ms_per_step": dt / args.steps * 1e3,
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u64",
            "data": ("synthetic: real 64-bit range proofs of random values made by the GPU prover "
                     "(generate_range_proof semantics, seeded randomness); generators per "
                     "complete_bulletproof_test.cu:33-109") if args.proofs == "prover" else
                    "synthetic (seeded proof-shaped inputs, a=[t], b=[1], c=t; generators per "
                    "complete_bulletproof_test.cu:33-109)",
            "config": {"workload": f"batch {B} x {n}-bit range-proof verify per GPU (BASELINE configs[1])",
                       "batch_per_gpu": B, "n": n, "semantics": "cuda_range_proof_verify (crv:82)",
                       "parallelism": f"independent proof shards x{world}", "mode": args.mode,
                       "pipeline_depth": pipe.depth if pipe else None, "pipelines": len(pipes) or None,
                       "prefix_tables": prefix,
                       "proof_bytes": proof_bytes(n, 1), "passes_in_warmup_batch": passes_warm},
            "roofline": roofline, "valu_roofline": valu_roofline, "cpu_baseline": cpu, "msm": msm, "ipa": ipa, "prove": prove,
            "sharded_2p16": sharded, "host_api": host_api,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()   # the other ranks wait out rank 0's single-GPU legs, then all leave together
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
