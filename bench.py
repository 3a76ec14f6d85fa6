"""bench.py — batched 64-bit range-proof verification on MI355X (BASELINE.json metric).

  python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B] [--n 64]
  python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
      --master-port P bench.py --gpus N --steps K --warmup W

--gpus N is N ranks: without a launcher, bench.py starts torch.distributed.run on itself as a
child process (before touching the GPU) and exits with its status; under a launcher WORLD_SIZE
must equal N.  The line carries world_size (from torch.distributed), each rank's device PCI
address and the verdict digest of its own batches (`ranks`).

One step = cuda_range_proof_verify semantics (crv:82) over one batch of B = 1024 synthetic
64-bit proofs already resident in HBM (BASELINE configs[1]); every rank verifies its own
batches (weak scaling, no data-path collective: proofs are independent).  K steps are timed
between barrier + synchronize on both sides; the max over ranks is the step time.

Extra fields on the JSON line:
  roofline     SURVEY 8(d) algorithmic bytes per step / ms_per_step vs HBM peak (the path is
               VALU-integer bound), PMC traffic per launch; valu_roofline beside it;
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
import statistics
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: 8.0 TB/s spec
# --prefix-bits default (tests/test_gpu_fullsize.py runs the same width): the smallest width within
# 0.5 % of the best measured (profiles/ab/r05a_prefix_sweep.json, one MI355X, median of 2 runs each:
# K 0 181.5 K, 16 188.0 K, 18 189.2 K, 20 190.0 K, 21 190.7 K, 22 191.0 K, 23 191.6 K verifies/s);
# K = 21 takes 34.9 GB of the 288 GB HBM (K = 23: 139.6 GB)
DEFAULT_PREFIX_BITS = 21
FE_B, GE_B = 32, 128


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200,
                    help="timed ticks per region (the sync at each end of a region costs about one tick's "
                         "tail: 50 ticks read 190.4 K, 2000 ticks 191.4 K)")
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
    ap.add_argument("--prove-streams", type=int, default=4,
                    help="HIP streams prover batches rotate over (4: 466-468 K vs 460-465 K with 2, "
                         "profiles/ab/r04n_prove_schedules.txt)")
    ap.add_argument("--no-prove", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--cpu-procs", type=int, default=0,
                    help="processes for the parallel CPU baseline (0: the job's CPU share, see cpu_share)")
    ap.add_argument("--no-msm", action="store_true")
    ap.add_argument("--proofs", choices=["prover", "synthetic"], default="prover",
                    help="verify inputs: proofs made by the GPU prover from random 64-bit values (default) "
                         "or proof-shaped random data")
    ap.add_argument("--prefix-bits", type=int, default=DEFAULT_PREFIX_BITS,
                    help="fixed-base prefix tables of the generators (hipbp_pipeline_prefix_tables; "
                         "0 = off): one-time setup, same bits (21: 34.9 GB at n = 64, within 0.5 %% of 23's "
                         "139.6 GB, profiles/ab/r05a_prefix_sweep.json)")
    ap.add_argument("--table-legs", default="0,16",
                    help="prefix-table widths timed beside the headline on the same batches (`prefix_legs`: "
                         "0 = the reference's plain double-and-add with no precompute); '' skips them")
    ap.add_argument("--shard-total", type=int, default=1 << 16, help="configs[4]: proofs in the sharded batch")
    ap.add_argument("--shard-batch", type=int, default=0,
                    help="configs[4]: proofs per pipeline push (0: auto from the rank's shard size)")
    ap.add_argument("--no-shard", action="store_true")
    ap.add_argument("--shard-defer", type=int, default=1,
                    help="configs[4]: split stage 0 in the shard's pipelines (hipbp_pipeline_defer_msm: the MSM "
                         "terms beside the fold rounds, so the drain overlaps them); same bits")
    ap.add_argument("--shard-stagger", type=int, default=0,
                    help="configs[4]: each push's stream waits for the previous push's pipeline to finish this many "
                         "more ticks (0: all pushes start together)")
    ap.add_argument("--shard-lockstep", action="store_true",
                    help="configs[4]: no pipeline starts its stage-0 tick before every pipeline's first push (challenges "
                         "+ lane sort) is done")
    ap.add_argument("--host-count", type=int, default=32768, help="proofs per host-struct API call")
    ap.add_argument("--no-host", action="store_true")
    ap.add_argument("--no-check", action="store_true", help="skip the headline self-check (verify_check)")
    ap.add_argument("--no-h2d", action="store_true", help="skip the H2D-inclusive headline (with_h2d)")
    ap.add_argument("--no-repeats", action="store_true", help="skip the 5 repeated timed regions (repeats)")
    ap.add_argument("--rehearse", action="store_true",
                    help="exercise the N>1 path on one GPU (all ranks on cuda:0, gloo collectives); not a measurement")
    return ap.parse_args()


TASK_B = GE_B + FE_B + GE_B   # one scalar-mult task: point + scalar in, term out


def verify_bytes(n):
    """SURVEY §8(d) algorithmic bytes of one n-bit verify: V + (V, A, S, T1, T2) + (taux, mu, t) +
    (n, c, L_len, x) + a, b (n entries each) + L, R (log2 n each) = 944 + 64 n + 256 log2 n
    (6,576 B at n = 64), plus 1 B of verdict out."""
    Lr = n.bit_length() - 1
    return 944 + 64 * n + 256 * Lr + 1


def gens_bytes(n):
    """the generators G, H (n points each) + g, h, read once per batch per GPU (16,640 B at n = 64)."""
    return 2 * n * GE_B + 2 * GE_B


def alg_bytes(kernel, B, n):
    """SURVEY §8(d) algorithmic HBM bytes of one batch of B verifies (the work one pipeline tick of
    `kernel` does in steady state): B x 6,577 B + 16,640 B at n = 64."""
    if kernel == "k_terms":
        return B * verify_bytes(n) + gens_bytes(n)
    return None


def traffic_model(B, n, prefix_bits):
    """Where k_terms' HBM bytes beyond the algorithmic ones come from (per tick of B verifies): every
    scalar multiplication writes its 128-B term and a later region reads it back (plus its 32-B
    scalar); each fixed-base one gathers one 128-B prefix-table entry; the lane-reduced MSM trees
    fold 2 x (n - 1) adds of 3 points in place.  A model to read the PMC total against, not a
    measurement."""
    sm = sm_per_verify(n)
    fixed = 4 * n + 2   # the two MSMs, fold round 0, t*h, c*Q start from the tables
    return {"terms_written_and_read": B * sm * (2 * GE_B + FE_B),
            "prefix_table_gathers": B * fixed * GE_B if prefix_bits else 0,
            "msm_lane_trees": B * 2 * (n - 1) * 3 * GE_B,
            "proof_and_generators": alg_bytes("k_terms", B, n)}


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
    """One process of the CPU baseline: verify proofs lo, lo+1, ... (cycling within [lo, hi)) with
    the reference build for `seconds`, starting at wall time `start_at` (the parallel run's workers
    all start together once every one of them has loaded, so their loops overlap)."""
    n, lo, hi, seconds, start_at = args
    from oracle import pyoracle
    R = pyoracle.Reference()
    G, H = R.base_points(n, 1), R.base_points(n, 2)
    g, h = R.gh()
    s, heads = _cpu_sample(n, hi)
    if start_at:
        time.sleep(max(0.0, start_at - time.time()))
    done, t0 = 0, time.perf_counter()
    while True:
        p = lo + done % (hi - lo)
        R.cuda_range_proof_verify(dict(head=heads[p], V=s["V"][p], a=s["a"][p], b=s["b"][p], L=s["L"][p],
                                       R=s["R"][p]), n, G, H, g, h)
        done += 1
        if time.perf_counter() - t0 > seconds:
            break
    return done, time.perf_counter() - t0


def cpu_share():
    """(nproc, affinity, used): the host's logical CPUs, the CPUs this process may run on, and the
    worker count the parallel baseline uses — the job's CPU share (OMP_NUM_THREADS, which the GPU
    box sets to the one-GPU share) when set, else the affinity set."""
    nproc = os.cpu_count() or 1
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = nproc
    omp = os.environ.get("OMP_NUM_THREADS")
    used = min(aff, int(omp)) if omp and omp.isdigit() and int(omp) > 0 else aff
    return nproc, aff, used


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
    done, dt = _cpu_worker((n, 0, 512, seconds, 0))
    out = {"value": done / dt, "unit": "verifies/s", "cores": 1, "kind": "reference",
           "sample": f"{done} synthetic {n}-bit proofs, the reference's cuda_range_proof_verify (oracle/_ref), "
                     f"1 thread, {dt:.1f} s", "cpu": cpu_model()}
    nproc, aff, used = cpu_share()
    procs = procs if procs > 0 else used
    out["nproc"], out["affinity_cpus"] = nproc, aff
    if procs > 1:
        import multiprocessing as mp
        per, par_s = 16, max(2.0, seconds / 4)
        with mp.get_context("spawn").Pool(procs) as pool:
            start_at = time.time() + 4.0 + 0.05 * procs   # after every worker has imported and loaded
            res = pool.map(_cpu_worker, [(n, k * per, (k + 1) * per, par_s, start_at) for k in range(procs)])
        tot = sum(r[0] for r in res)
        out["parallel"] = {"value": sum(r[0] / r[1] for r in res), "unit": "verifies/s", "cores": procs,
                           "nproc": nproc, "affinity_cpus": aff,
                           "sample": f"{tot} proofs over {procs} concurrent processes ({par_s:.1f} s each, started "
                                     f"together; one per CPU of the job's share: the host has {nproc} logical "
                                     f"CPUs, {aff} in this process's affinity set)"}
    return out


def configs0_leg(reps=15):
    """BASELINE configs[0]: the reference's own main() flow (complete_bulletproof_test.cu:65-310:
    one 16-bit proof of value 42 generated and verified both ways, the out-of-range proof, the
    field-op benchmark) on this host, timed as the process it is: oracle/_ref's CPU twin (the GPU
    symbols host-emulated: the reference CPU path end to end) `reps` times, median wall, plus the
    verify times main() prints itself; and once as the drop-in binary on our library (the same
    main() with cuda_* on the GPU, HIP initialisation included).  The driver ends in its own
    undefined behaviour (SIGSEGV at complete_bulletproof_test.cu:305, tests/test_dropin.py) after
    all of its output; that exit status is recorded, not treated as an error.  Runs before this
    process touches the GPU (children only)."""
    import re
    import subprocess
    ref = os.path.join(ROOT, "oracle", "_ref")
    cpu_bin, hip_bin = (os.path.join(ref, f"complete_bulletproof_test_{k}") for k in ("cpu", "hip"))
    if not os.path.exists(cpu_bin):
        return None

    def run(path):
        env = dict(os.environ, BP_RAND_SEED="1")
        t0 = time.perf_counter()
        p = subprocess.run(["stdbuf", "-oL", path], capture_output=True, text=True, timeout=300, env=env)
        wall = time.perf_counter() - t0
        grab = lambda k: [float(x) for x in re.findall(k + r" Time: ([0-9.]+) seconds", p.stdout)]
        return {"wall_s": wall, "rc": p.returncode, "cuda_verify_s": grab("CUDA Verification"),
                "cpu_verify_s": grab("CPU Verification"),
                "ok": "CUDA Verification result: SUCCESS" in p.stdout and "CPU Verification result: SUCCESS" in p.stdout
                      and "FAILED (CORRECT)" in p.stdout}
    runs = [run(cpu_bin) for _ in range(reps)]
    out = {"workload": "BASELINE configs[0]: complete_bulletproof_test main(), 16-bit proof of value 42, "
                       "generate + cuda_range_proof_verify + range_proof_verify + out-of-range proof + field-op "
                       "benchmark", "unit": "s per run",
           "cpu_path": {"value": statistics.median(r["wall_s"] for r in runs), "runs": reps,
                        "min": min(r["wall_s"] for r in runs),
                        "verify_s_median": statistics.median(r["cuda_verify_s"][0] for r in runs if r["cuda_verify_s"]),
                        "range_proof_verify_s_median": statistics.median(r["cpu_verify_s"][0] for r in runs
                                                                         if r["cpu_verify_s"]),
                        "all_ok": all(r["ok"] for r in runs), "exit_status": sorted({r["rc"] for r in runs}),
                        "binary": "oracle/_ref/complete_bulletproof_test_cpu (reference sources, GPU symbols "
                                  "host-emulated)", "cores": 1}}
    if os.path.exists(hip_bin):
        h = run(hip_bin)
        out["dropin_gpu"] = {"value": h["wall_s"], "cuda_verify_s": h["cuda_verify_s"], "ok": h["ok"],
                             "exit_status": h["rc"],
                             "binary": "oracle/_ref/complete_bulletproof_test_hip (the same main() on "
                                       "libcudabulletproof_hip.so; wall includes HIP runtime start-up; its "
                                       "printed times are the driver's clock(), process CPU time)"}
    out["dropin_latency"] = dropin_latency()
    return out


def dropin_proof_file(path, n=16, i=0):
    """proof.bin for tests/dropin_latency.c: reference proof i of tests/golden/proofs_n{n}.npz
    (complete_bulletproof_test.cu's generators; proof 0 is its value-42 proof)."""
    d = np.load(os.path.join(ROOT, "tests", "golden", f"proofs_n{n}.npz"))
    h = d["head"][i]
    with open(path, "wb") as f:
        f.write(np.array([n, d["a"].shape[1], d["L"].shape[1]], np.uint64).tobytes())
        for a in (d["G"], d["H"], d["g"], d["h"], d["V"][i], h[16:80], h[80:100], d["a"][i], d["b"][i], d["L"][i],
                  d["R"][i]):
            f.write(np.ascontiguousarray(a, np.uint64).tobytes())
    return bool(d["ok_cuda"][i])


def build_dropin_latency():
    """Compile tests/dropin_latency.c against the product library into build/ (gcc, seconds)."""
    import subprocess
    out = os.path.join(ROOT, "build", "dropin_latency")
    src = os.path.join(ROOT, "tests", "dropin_latency.c")
    lib = os.path.join(ROOT, "cudabulletproof_amd", "libcudabulletproof_hip.so")
    if os.path.exists(out) and os.path.getmtime(out) >= max(os.path.getmtime(src), os.path.getmtime(lib)):
        return out
    os.makedirs(os.path.dirname(out), exist_ok=True)
    subprocess.check_call(["gcc", "-O2", "-I" + os.path.join(ROOT, "include"), src,
                           "-L" + os.path.dirname(lib), "-lcudabulletproof_hip",
                           "-Wl,-rpath," + os.path.dirname(lib), "-o", out])
    return out


def dropin_latency(ns=(16, 64), warm=20):
    """Wall-clock latency of the drop-in cuda_range_proof_verify, one reference proof per call, in
    a fresh process per n (tests/dropin_latency.c: the HIP runtime's start-up, the first call, the
    median warm call), beside the reference CPU path's per-verify time.  Children only: this
    process has not touched the GPU."""
    import subprocess
    import tempfile
    try:
        exe = build_dropin_latency()
    except (OSError, subprocess.CalledProcessError) as e:
        return {"error": str(e)}
    res = {}
    with tempfile.TemporaryDirectory() as tmp:
        for n in ns:
            pf = os.path.join(tmp, f"proof{n}.bin")
            want = dropin_proof_file(pf, n)
            p = subprocess.run([exe, pf, str(warm)], capture_output=True, text=True, timeout=300)
            try:
                r = json.loads(p.stdout.strip().splitlines()[-1])
                r["matches_reference_verdict"] = r["verdict"] == want
            except (ValueError, IndexError):
                r = {"rc": p.returncode, "stderr": p.stderr[-500:]}
            res[f"n{n}"] = r
    res["harness"] = "tests/dropin_latency.c (CLOCK_MONOTONIC; one reference proof of tests/golden/proofs_n*.npz)"
    return res


def oracle_sample(n, B, seed, count=64, procs=0):
    """The checker for the headline's self-check (bench `verify_check`): the first `count` proofs of
    the bench's batch 0 made by the CPU restatement's prover from the same inputs
    (synth.prove_inputs(B, n, seed) rows 0..count-1) and verified by it (crv:82 semantics): their
    verdicts and IPA points P.  Test infrastructure, run before the GPU is touched, in worker
    processes over the job's CPU share."""
    count = min(count, B)
    procs = max(1, min(procs or cpu_share()[2], 16, count))
    cuts = [count * k // procs for k in range(procs + 1)]
    jobs = [(n, B, seed, a, b) for a, b in zip(cuts[:-1], cuts[1:]) if b > a]
    if len(jobs) == 1:
        parts = [_oracle_sample_rows(jobs[0])]
    else:
        import multiprocessing as mp
        with mp.get_context("spawn").Pool(len(jobs)) as pool:
            parts = pool.map(_oracle_sample_rows, jobs)
    return {k: np.concatenate([p[k] for p in parts]) for k in ("ok", "P", "A")}


def _oracle_sample_rows(args):
    """oracle_sample's rows [lo, hi): the restatement's prover + verifier (one worker process)."""
    n, B, seed, lo, hi = args
    from oracle import pyoracle
    from cudabulletproof_amd import synth
    O = pyoracle.Oracle()
    G, H = O.base_points(n, 1), O.base_points(n, 2)
    g, h = O.gh()
    pi = synth.prove_inputs(B, n, seed=seed)
    oks, Ps, heads = [], [], []
    for p in range(lo, hi):
        sLR = np.concatenate([pi["sL"][p].view(np.uint8).reshape(n, 32), pi["sR"][p].view(np.uint8).reshape(n, 32)],
                             axis=1)
        pr = O.generate_range_proof(pi["v"][p].view(np.uint8), pi["gamma"][p].view(np.uint8), sLR,
                                    pi["rnd"][p].view(np.uint8).reshape(4, 32), n, G, H, g, h)
        ok, P, _, _, _ = O.cuda_range_proof_verify(pr["head"], pr["V"], n, pr["a"], pr["b"], pr["L"], pr["R"],
                                                   G, H, g, h)
        oks.append(ok)
        Ps.append(P)
        heads.append(pr["head"])
    return {"ok": np.array(oks, np.uint8), "P": np.stack(Ps), "A": np.stack([hh[16:32] for hh in heads])}


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


def rooflines(dom, B, n, steps, launches, avg_ms, dt, kern_ms, pcfg, npipes):
    """`roofline` (HBM, as the contract asks) and `valu_roofline` (the binding resource) for the
    dominant kernel.  HBM: SURVEY §8(d) algorithmic bytes of the timed region's batches / the
    region's wall time (one step = one k_terms launch of one batch; the launches of the two
    pipelines overlap, so the per-launch HIP-event rate goes beside it as `per_launch_overlapped`,
    measured on the library's streams); `traffic` = the PMC bytes per
    launch (profiles/pmc_traffic.json, collected on this configuration) with its ratio to the
    algorithmic bytes and a breakdown model.  VALU: `frac` = VALUBusy (PMC: the fraction of cycles
    in which the SIMDs issued VALU work); beside it the region's issue rate (SQ_INSTS_VALU per
    launch x launches / wall time), the cycles per instruction per SIMD that rate means at the PMC
    clock and at the shader clock measured under this load (profiles/clock/), and the rates of
    k_terms' point-op loops run alone (profiles/valu_step_roof.json)."""
    per_batch = alg_bytes(dom, B, n)
    per_launch = per_batch * steps / launches if per_batch else None
    achieved = (per_launch / (avg_ms * 1e-3)) / 1e9 if per_launch else None
    agg = per_batch * steps / dt / 1e9 if per_batch else None
    traffic = pmc(dom, "bytes_per_launch", pcfg)
    model = traffic_model(B, n, pcfg["prefix_bits"]) if dom == "k_terms" else None
    roofline = {
        "bound": "hbm", "kernel": dom, "achieved": agg, "peak": HBM_PEAK_GBS, "unit": "GB/s",
        "frac": agg / HBM_PEAK_GBS if agg else None, "traffic": traffic,
        "achieved_rule": "SURVEY 8(d) algorithmic bytes of the timed steps / the timed region's wall time "
                         "(= per step / ms_per_step): one step is one k_terms launch of one batch, and with two "
                         "pipelines the launches overlap, so a launch's own duration is not a per-step time",
        "alg_bytes_per_step": per_batch, "alg_bytes_per_launch": per_launch,
        "alg_bytes_rule": f"SURVEY 8(d): {verify_bytes(n) - 1} B per verify (944 + 64n + 256 log2 n) + 1 B verdict, "
                          f"x {B} verifies + {gens_bytes(n)} B generators per batch",
        "traffic_over_alg": traffic / per_launch if traffic and per_launch else None,
        "traffic_model_bytes": model,
        "per_launch_overlapped": {
            "achieved": achieved, "frac": (achieved / HBM_PEAK_GBS) if achieved else None, "avg_launch_ms": avg_ms,
            "note": "bytes per launch / the launch's own HIP-event duration, which includes the other pipeline's "
                    "overlapping launch (a lower bound of the per-kernel rate)"},
        "avg_launch_ms": avg_ms, "launches": launches, "concurrent_pipelines": npipes or None,
        "rocprof_avg_launch_ms": pmc(dom, "rocprof_avg_ms", pcfg),
        "kernel_ms_share": {k: round(v / sum(kern_ms.values()), 4) for k, v in kern_ms.items()},
        "binding": "VALU integer issue (not HBM, not MFMA): see DESIGN.md and valu_roofline",
    }
    vi = pmc(dom, "valu_instr_per_launch", pcfg)
    busy = pmc(dom, "valu_busy_pct", pcfg)
    alg_vi = alg_valu_per_verify(n, pcfg["prefix_bits"]) * B if dom == "k_terms" else None
    clk = pmc(dom, "eff_clock_ghz", pcfg)
    vagg = vi * launches / dt if vi else None   # all launches of the timed region / its wall time
    loops = step_roof()
    clk_loaded = loaded_clock_mhz()
    # the products the formulas need, per second of the timed region, against the guide's nominal
    # wave64 issue of every SIMD (1024 SIMDs x the loaded shader clock / 2 cycles per instruction):
    # a roof that is not the kernel's own measured issue rate
    nominal = 1024 * clk_loaded * 1e6 / 2 if clk_loaded else None
    frac_nominal = alg_vi * launches / dt / nominal if alg_vi and nominal else None
    frac_alg = alg_vi / vi * busy / 100 if alg_vi and vi and busy else None
    # scalars the driver's parsed copy of the line keeps (it drops nested objects)
    roofline["kernel_ms_per_step"] = avg_ms / npipes if npipes else avg_ms
    roofline["frac_per_launch_overlapped"] = achieved / HBM_PEAK_GBS if achieved else None
    roofline["valu_frac_busy"] = busy / 100 if busy else None
    roofline["valu_frac_alg"] = frac_alg
    roofline["valu_frac_nominal_issue"] = frac_nominal
    valu_roofline = {
        "kernel": dom, "unit": "wave64 VALU instr/s", "frac": busy / 100 if busy else None,
        "frac_source": "VALUBusy (rocprofv3 PMC on this configuration, profiles/pmc_traffic.json): the share of "
                       "cycles the SIMDs spend issuing VALU work",
        "instr_per_launch": vi, "achieved_aggregate": vagg, "eff_clock_ghz": clk,
        "cycles_per_instr_per_simd_aggregate": 1024 * clk * 1e9 / vagg if vagg and clk else None,
        "cycles_per_instr_per_simd_serialized": pmc(dom, "serial_cycles_per_instr_per_simd", pcfg),
        "isolated_loops": {k: {"Ginstr_per_s": v["Ginstr_per_s"], "cycles_per_instr_per_simd":
                               v["cycles_per_instr_per_simd"]} for k, v in loops["kernels"].items()} if loops else None,
        "isolated_loops_source": "profiles/valu_step_roof.json (tools/ubench_step.hip: k_terms' point-op loops "
                                 "from registers + LDS at its occupancy)",
        "valu_utilization_pct": pmc(dom, "valu_utilization_pct", pcfg), "pmc_config": pcfg,
        "loaded_clock_mhz": clk_loaded,
        "cycles_per_instr_per_simd_loaded_clock": 1024 * clk_loaded * 1e6 / vagg if vagg and clk_loaded else None,
        "frac_nominal_issue": frac_nominal,
        "frac_nominal_issue_rule": "minimum product VALU per launch x launches / the timed region's wall time, over "
                                   "1024 SIMDs x loaded shader clock / 2 cycles (the guide's nominal wave64 issue)",
        "loaded_clock_source": "profiles/clock/*.json (tools/clock_watch.sh: rocm-smi shader clock, median over the "
                               "headline's loaded samples; not throttled at ~1.25 kW): the issue interval this run's "
                               "aggregate VALU rate means at that clock",
        "frac_alg": frac_alg,
        "alg_product_valu_per_launch": alg_vi,
        "frac_alg_rule": "minimum product VALU per launch (2 VALU per 32x32 limb product: 464 products per doubling "
                         "with its squares, 512 per add with Z2 = 1; point ops per verify from bench.point_ops_model "
                         "at this prefix width) / measured SQ_INSTS_VALU per launch x VALUBusy: the share of "
                         "the SIMDs' issue cycles spent on the products the reference's formulas require",
    }
    return roofline, valu_roofline


def point_ops_model(n, K):
    """Expected point operations of one verify (crv:82 semantics), for scalars uniform below 2^255:
    the 4n + 2 fixed-base scalar-mults (the two MSMs, fold round 0, t*h, c*Q) start after a K-bit
    prefix-table entry (256 - K doublings, (255 - K) / 2 adds expected); the other sm_per_verify(n) -
    (4n + 2) (fold rounds >= 1, a0 G', b0 H') run all 256 bits minus ~1 leading zero (254
    doublings, 127 adds expected).  A model: the exact counts depend on the proofs' scalars."""
    fixed = 4 * n + 2
    other = sm_per_verify(n) - fixed
    dbl = fixed * (256 - K) + other * 254 if K else (fixed + other) * 254
    add = fixed * (255 - K) / 2 + other * 127 if K else (fixed + other) * 127
    return dbl, add


# 32x32-bit limb products per point operation the reference's formulas need at minimum: a doubling
# (ge25519_add(r, r), curve25519_ops.cu:406) = 4 squares (36 products) + 5 general products (64);
# an add with Z2 = 1 (the generators and normalized points) = 8 general products (Z1 Z2 = Z1)
PRODUCTS_DBL, PRODUCTS_ADD = 4 * 36 + 5 * 64, 8 * 64


def alg_valu_per_verify(n, K):
    """Minimum product VALU of one verify in wave64 instructions: 2 VALU per 32x32 product (one
    v_mad_u64_u32 + one carry count), per the point_ops_model, / 64 lanes."""
    dbl, add = point_ops_model(n, K)
    return 2 * (dbl * PRODUCTS_DBL + add * PRODUCTS_ADD) / 64


def loaded_clock_mhz():
    """Median shader clock under the headline's load, from the latest round's profiles/clock/clock_<tag>.json
    (ordered by file name, i.e. by round tag: a checkout gives every file the same mtime)."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "clock", "clock_*.json")))
    try:
        return float(json.load(open(files[-1]))["sclk_mhz_median_loaded"]) if files else None
    except (OSError, ValueError, KeyError):
        return None


def step_roof():
    try:
        return json.load(open(os.path.join(ROOT, "profiles", "valu_step_roof.json")))
    except (OSError, ValueError):
        return None


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


def headline_check(B, n, pipes, streams, batch, Gd, Hd, hd, sample):
    """Self-check of the headline configuration, outside the timed region: batch 0 through the timed
    pipeline (its generator set's prefix tables, the bench's pipelines and streams) and through a
    fresh table-free pipeline must give the same verdicts and IPA points P bit for bit, and their
    first proofs must match the CPU restatement's (oracle_sample: the same prover inputs proved and
    verified on the CPU)."""
    import torch
    import cudabulletproof_amd as bp
    dev = batch.V.device
    outs = []
    plain = bp.VerifyPipeline(B, n, Gd, Hd, hd, stream=streams[0])
    for pl in (pipes[0], plain):
        ok = torch.zeros(B, dtype=torch.uint8, device=dev)
        P = torch.zeros(B, 16, dtype=torch.int64, device=dev)
        pl.push(batch, ok, P_out=P)
        pl.flush()
        torch.cuda.synchronize(dev)
        outs.append((ok, P))
    plain.close()
    (ok, P), (ok0, P0) = outs
    d = lambda t: hashlib.sha256(t.cpu().numpy().tobytes()).hexdigest()[:16]
    res = {"batch": 0, "proofs": B, "passes": int(ok.sum().item()), "verdicts_sha256": d(ok), "P_sha256": d(P),
           "tables_equal_plain": bool(torch.equal(ok, ok0) and torch.equal(P, P0))}
    if sample is not None:
        k = len(sample["ok"])
        res["oracle_sample"] = k
        res["proofs_match_oracle_prover"] = bool(np.array_equal(batch.A[:k].cpu().numpy().view(np.uint64),
                                                                sample["A"]))
        res["matches_oracle_sample"] = bool(np.array_equal(ok[:k].cpu().numpy(), sample["ok"]) and
                                            np.array_equal(P[:k].cpu().numpy().view(np.uint64), sample["P"]))
    return res


def h2d_leg(args, dev, pipes, batches, steps, want_oks=None):
    """The headline with the per-batch proof H2D inside the timed region (SURVEY §8(d) timing rule):
    every step copies its batch (B proofs in the flat wire format, ≈2.3 KB each) from pinned host
    memory into one of a few device staging batches on a copy stream, and the pipeline's stream
    waits for that copy before the tick; a staging batch is overwritten only after the tick that
    consumed it.  Every step writes its own verdict slice; after the flush each step's verdicts must
    equal the resident headline's for the same batch (`want_oks`, `verdicts_match_resident`).
    PCIe-inclusive: reported beside `value`, never as it."""
    import torch
    import cudabulletproof_amd as bp
    F = bp.RangeProofBatch.FIELDS
    # one contiguous wire-format buffer per batch (fields back to back, 32-byte aligned), so a step
    # is ONE pinned-host -> HBM copy (the fields as separate copies were 14 small transfers per step)
    shapes = [(f, getattr(batches[0], f).shape, getattr(batches[0], f).dtype) for f in F]
    sizes = [getattr(batches[0], f).numel() * getattr(batches[0], f).element_size() for f in F]
    offs = np.cumsum([0] + sizes)
    nbytes = int(offs[-1])

    def views(buf):
        return {f: buf[offs[i]:offs[i + 1]].view(dt).view(shp) for i, (f, shp, dt) in enumerate(shapes)}

    host = []
    for b in batches:
        hb = torch.empty(nbytes, dtype=torch.uint8).pin_memory()
        for f, t in views(hb).items():
            t.copy_(getattr(b, f).cpu())
        host.append(hb)
    AHEAD = int(os.environ.get("BENCH_H2D_AHEAD", "2"))   # copies issued this many steps before their tick
    nst = 2 * len(pipes) + 2 + AHEAD
    stage = [torch.empty(nbytes, dtype=torch.uint8, device=dev) for _ in range(nst)]
    stage_views = [views(sb) for sb in stage]
    cst = torch.cuda.Stream(dev)
    fill = (pipes[0].depth - 1) * len(pipes)   # fill, as the headline
    # one verdict slice per step: a batch writes its verdicts depth - 1 ticks after its push, so a
    # ring of staging-sized ok buffers would be shared by batches still in flight
    oks = torch.zeros(fill + steps, args.batch, dtype=torch.uint8, device=dev)
    consumed = [None] * nst

    # each batch's copy is issued AHEAD steps before its tick (a copy can queue behind a running
    # tick's blocks; issued with its own tick it delayed that tick): one box, 50 steps: 162-176 K
    # verifies/s issued with the tick, 182-184 K issued 2, 4 or 6 steps ahead
    issued = {}

    def copy(g):
        j = g % nst
        with torch.cuda.stream(cst):
            if consumed[j] is not None:   # the push that last used staging j (g - nst < g - AHEAD)
                cst.wait_event(consumed[j])
            stage[j].copy_(host[g % len(host)], non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(cst)
        issued[g] = ev

    def step(g, last):
        for a in range(g, min(g + AHEAD, last) + 1):
            if a not in issued:
                copy(a)
        j = g % nst
        pl = pipes[g % len(pipes)]
        pl_stream = pl.stream if pl.stream is not None else torch.cuda.default_stream(dev)
        pl_stream.wait_event(issued.pop(g))
        pl.push(bp.RangeProofBatch(args.n, **stage_views[j]), oks[g])
        done = torch.cuda.Event()
        done.record(pl_stream)
        consumed[j] = done

    for g in range(fill):
        step(g, fill - 1)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for g in range(fill, fill + steps):
        step(g, fill + steps - 1)
    torch.cuda.synchronize(dev)
    dt = time.perf_counter() - t0
    for pl in pipes:
        pl.flush()
    torch.cuda.synchronize(dev)
    match = None
    if want_oks is not None:   # step g verified host batch g % len(host), the headline's batch g % nb
        got = oks.cpu()
        match = all(torch.equal(got[g], want_oks[g % len(host)].cpu()) for g in range(fill + steps))
    return {"metric": "64-bit range-proof verifies/sec, per-batch proof H2D inside the timed region",
            "verdicts_match_resident": match,
            "value": args.batch * steps / dt, "unit": "verifies/s", "ms_per_step": dt / steps * 1e3,
            "bytes_h2d_per_step": nbytes, "copies_per_step": 1, "copy_ahead_steps": AHEAD, "h2d_GBps": nbytes * steps / dt / 1e9, "staging_batches": nst,
            "note": "pinned host -> HBM on a copy stream overlapped with the ticks; PCIe-inclusive, never `value`"}


def shard_push_batch(args, shard_size, npipe):
    """Proofs per push for a rank's shard.  A pushed batch completes depth - 1 ticks after its push,
    and its last ticks (fold rounds 3..5, final terms, final assembly) are latency-bound, so a small
    shard (8192 proofs per rank at N = 8) goes through in one push per pipeline of at most 4096
    proofs: the two pipelines' latency-bound drain ticks then run side by side (tools/shard_probe.py,
    profiles/NOTES.md §5: 4096+4096 169.4 K, 2048 x 4 162.5 K, decreasing schedules 150-156 K)."""
    if args.shard_batch > 0:
        return args.shard_batch
    per = -(-shard_size // npipe)
    Bs = args.batch
    while Bs < per and Bs < 4096:
        Bs *= 2
    return Bs


def shard_leg(args, dev, world, rank, pipes, gens, G, H, g, h, streams=None):
    """configs[4]: ONE batch of 2^16 64-bit proofs (1024 x 4 distinct proofs, tiled: the kernels do
    not dedupe) split into equal contiguous shards over the ranks (shard.shard_bounds).  Each rank
    verifies its shard through its pipelines; the pass counts meet in one all_reduce(SUM) and the
    2^16 verdict bytes in one all_gather over RCCL (every rank ends with all verdicts).  Timed
    from a barrier to the end of the collectives (pipeline fill and drain included), max over ranks,
    after one untimed pass; the median of 5 timed passes; strong scaling: the same 2^16 proofs
    whatever N."""
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
    defer = False
    if args.shard_defer:   # the split stage 0 for the shard's batches, where the C ABI accepts it
        try:
            for pp in pipes:
                pp.defer_msm(True)
            defer = True
        except bp.BulletproofError:   # (n < 4 or above the lane-tree limit: the unsplit pipeline)
            for pp in pipes:
                pp.defer_msm(False)
    try:
        return _shard_run(args, dev, world, B, n, total, lo, hi, tiles, pipes, Bs, defer)
    finally:
        if defer:   # the headline pipelines get it back off whatever happened
            for pp in pipes:
                pp.defer_msm(False)
        for pp in own:
            pp.close()


def _shard_run(args, dev, world, B, n, total, lo, hi, tiles, pipes, Bs, defer):
    import torch
    import torch.distributed as dist
    import cudabulletproof_amd as bp
    from cudabulletproof_amd import shard

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

    def run_once():
        ok.zero_()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for k, b in enumerate(batches):
            pp = pipes[k % len(pipes)]
            if args.shard_stagger and k > 0 and len(pipes) > 1:   # start after the previous push's first ticks
                prev = pipes[(k - 1) % len(pipes)]
                for _ in range(args.shard_stagger):
                    prev.push(None)
                ev = torch.cuda.Event()
                ev.record(prev.stream)
                pp.stream.wait_event(ev)
            pp.push(b, ok[offs[k]:offs[k + 1]])
        if args.shard_lockstep and len(pipes) > 1:   # every pipeline's next tick waits for every first push
            evs = []
            for pp in pipes:
                ev = torch.cuda.Event()
                ev.record(pp.stream)
                evs.append(ev)
            for i, pp in enumerate(pipes):
                for j, ev in enumerate(evs):
                    if i != j:
                        pp.stream.wait_event(ev)
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
        return time.perf_counter() - t0, passes, allv

    # one untimed pass (the new pipelines' first ticks, code-object loads), then 5 timed passes
    # (>= 5 repetitions, median): `value` is the median, max over ranks per pass;
    # every pass must give the same verdicts
    run_once()
    times, digests = [], set()
    for _ in range(5):
        dt, passes, allv = run_once()
        times.append(dt)
        digests.add(allv.cpu().numpy().tobytes())
    if world > 1:
        t = torch.tensor(times, dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        times = [float(x) for x in t.tolist()]
    dt = statistics.median(times)
    import hashlib as _h
    return {"metric": "2^16-proof 64-bit range-proof batch verify (BASELINE configs[4])", "value": total / dt,
            "push_batch": Bs, "defer_msm": defer, "passes_timed": len(times),
            "value_min": total / max(times),
            "value_max": total / min(times), "same_verdicts_every_pass": len(digests) == 1,
            "unit": "verifies/s", "proofs": total, "n_gpus": world, "scaling": "strong", "ms": dt * 1e3,
            "passes": int(passes.item()), "verdicts_sha256": _h.sha256(allv.cpu().numpy().tobytes()).hexdigest()[:16],
            "collectives": "all_reduce(SUM) of pass counts + all_gather of the verdict bytes (RCCL at N > 1)",
            "data": "1024 x 4 distinct GPU-prover proofs (rank-independent seeds), tiled to 2^16"}


def host_leg(args, batches, G, H, g, h):
    """The host-struct entry point hipbp_batch_range_proof_verify_host: an array of the reference's
    own RangeProof structs in host memory (cuda_range_proof_verify semantics per proof), so the
    rate includes packing, one H2D, the pipeline and one D2H (PCIe-inclusive; never `value`).
    Timed over calls after the first, which also builds the generator set's prefix tables
    (`first_call_ms`)."""
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
    t1 = time.perf_counter()
    call()   # the first call also builds the generator set's prefix tables the engine then keeps
    first_ms = (time.perf_counter() - t1) * 1e3
    reps = 2
    t1 = time.perf_counter()
    for _ in range(reps):
        call()
    dt = (time.perf_counter() - t1) / reps
    return {"metric": "64-bit range-proof verifies/sec, host RangeProof structs (PCIe-inclusive)",
            "value": count / dt, "unit": "verifies/s", "proofs": count, "ms": dt * 1e3, "passes": int(ok.sum()),
            "first_call_ms": first_ms, "n_gpus": 1, "entry_point": "hipbp_batch_range_proof_verify_host",
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
    # batches rotate over --prove-streams streams (default 4): one batch's latency-bound stages (T
    # terms, IPA rounds, chains) run under the other batches' term launches (each stream has its own
    # prover workspace in the engine)
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


def prefix_leg(args, dev, world, bits, batches, ref_oks, G, H, g, h, streams):
    """The headline configuration at another prefix-table width (`prefix_legs`): fresh pipelines on
    the same streams over the same resident batches, a generator set with `bits`-bit tables (none at
    0: every scalar-mult is the reference's full 256-bit double-and-add, cuda_bulletproof_kernels.cu:26-41),
    filled, then args.steps ticks timed between barrier + synchronize like `value` (max over ranks).
    The leg writes its own zeroed verdict buffers; the verdicts of every batch must equal the
    headline's (`verdicts_match_headline`; None when the leg pushed fewer than all the batches)."""
    import torch
    import torch.distributed as dist
    import cudabulletproof_amd as bp
    B, n, nb = args.batch, args.n, len(batches)
    oks = [torch.zeros_like(o) for o in ref_oks]
    gens = None
    torch.cuda.synchronize(dev)
    tb = time.perf_counter()
    if bits:
        gens = bp.Generators(n, G, H, g, h, prefix_bits=bits)
        torch.cuda.synchronize(dev)
    build_s = time.perf_counter() - tb
    npipe = max(1, args.pipes)
    pipes = [bp.VerifyPipeline(B, n, G, H, h, stream=streams[i]) for i in range(npipe)]
    try:
        if gens is not None:
            for pp in pipes:
                pp.use_gens(gens)
        step = lambda k: pipes[k % npipe].push(batches[k % nb], oks[k % nb])
        for k in range((pipes[0].depth - 1) * npipe):
            step(k)
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
        for pp in pipes:
            pp.flush()
        torch.cuda.synchronize(dev)
        pushed = (pipes[0].depth - 1) * npipe + args.steps
        same = all(torch.equal(o, r) for o, r in zip(oks, ref_oks)) if pushed >= nb else None
    finally:
        for pp in pipes:
            pp.close()
        if gens is not None:
            gens.close()
        torch.cuda.empty_cache()
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    return {"prefix_bits": bits, "value": B * args.steps * world / dt, "ms_per_step": dt / args.steps * 1e3,
            "steps": args.steps, "tables_GB": (2 * n + 2) * (1 << bits) * GE_B / 1e9 if bits else 0.0,
            "tables_build_s": build_s if bits else None, "verdicts_match_headline": same}


def kfd_gpu_count(sysfs="/sys/class/kfd/kfd/topology/nodes", dev_dri="/dev/dri", env=None):
    """GPUs this process could open, counted without the HIP runtime (the launcher parent must not
    bring it up): KFD topology nodes with SIMDs (CPU nodes have simd_count 0) whose render node
    /dev/dri/renderD<drm_render_minor> exists here (a container sees only the GPUs passed to it),
    capped by the visible-device lists HIP honours (HIP_ / ROCR_ / CUDA_VISIBLE_DEVICES).  None when
    the topology is absent (no amdgpu driver)."""
    env = os.environ if env is None else env
    try:
        nodes = sorted(os.listdir(sysfs))
    except OSError:
        return None
    count = 0
    for nd in nodes:
        props = {}
        try:
            for line in open(os.path.join(sysfs, nd, "properties")):
                k, _, v = line.strip().partition(" ")
                props[k] = v
        except OSError:
            continue
        if int(props.get("simd_count", "0") or 0) <= 0:
            continue
        minor = props.get("drm_render_minor")
        if minor is not None and not os.path.exists(os.path.join(dev_dri, f"renderD{minor}")):
            continue
        count += 1
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = env.get(var)
        if v is not None:
            count = min(count, len([x for x in v.split(",") if x.strip() and x.strip() != "-1"]))
    return count


def hip_mapped():
    """The HIP / HSA runtime libraries mapped into this process (/proc/self/maps), [] if none."""
    try:
        libs = {line.split()[-1] for line in open("/proc/self/maps") if len(line.split()) >= 6}
    except OSError:
        return []
    return sorted(os.path.basename(p) for p in libs if "libamdhip64" in p or "libhsa-runtime64" in p)


def rank_launch(args):
    """`--gpus N` means N ranks.  Under a launcher (WORLD_SIZE set) the world must be N.  Without
    one and N > 1, this process starts `torch.distributed.run --nproc-per-node N` on this script as
    a CHILD and returns its exit status; N larger than the visible GPUs is an error (--rehearse puts
    every rank on cuda:0).  This launcher never touches the GPU: no torch import, devices counted
    from the KFD topology (kfd_gpu_count).  Before the spawn it runs the CPU legs rank 0 would run
    at N = 1 (cpu_baseline, configs0: children and host code only) and hands their JSON to rank 0
    through a temp file (BENCH_CPU_LEGS), with whether a HIP runtime was mapped here up to the spawn.
    BENCH_LAUNCH_DRYRUN=1 prints that hand-over instead of spawning (tests/test_bench_helpers.py).
    Returns None when this process is a rank and should run the bench."""
    ws = os.environ.get("WORLD_SIZE")
    if ws is not None:
        if int(ws) != args.gpus:
            print(f"bench.py: --gpus {args.gpus} but the launcher started WORLD_SIZE={ws} ranks", file=sys.stderr)
            return 2
        return None
    if args.gpus <= 1:
        return None
    import socket
    import subprocess
    import tempfile
    have = kfd_gpu_count()
    if (have is None or have < args.gpus) and not args.rehearse:
        print(f"bench.py: --gpus {args.gpus} needs {args.gpus} GPUs, {have or 0} visible "
              f"(--rehearse runs every rank on cuda:0 with gloo)", file=sys.stderr)
        return 3
    legs = {"cpu_baseline": None, "configs0": None}
    if not args.no_cpu:
        legs["cpu_baseline"] = cpu_baseline(args.n, args.cpu_seconds, args.cpu_procs)
        legs["configs0"] = configs0_leg()
    legs["launcher"] = {"gpus_visible_kfd": have, "hip_mapped_before_spawn": hip_mapped(),
                        "note": "the torchrun parent: counted GPUs from /sys/class/kfd, ran the CPU legs, spawned"}
    fd, path = tempfile.mkstemp(prefix="bench_cpu_legs_", suffix=".json")
    with os.fdopen(fd, "w") as f:
        json.dump(legs, f)
    try:
        if os.environ.get("BENCH_LAUNCH_DRYRUN") == "1":
            print(json.dumps(dict(legs, hand_over=path)), flush=True)
            return 0
        with socket.socket() as s:   # a free rendezvous port on the loopback
            s.bind(("127.0.0.1", 0))
            port = s.getsockname()[1]
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
               "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
        return subprocess.call(cmd, env=dict(os.environ, BENCH_CPU_LEGS=path))
    finally:
        os.unlink(path)


def cpu_legs_handed_over():
    """The launcher parent's CPU legs (rank_launch), or None when this rank was not started by it."""
    path = os.environ.get("BENCH_CPU_LEGS")
    if not path:
        return None
    try:
        return json.load(open(path))
    except (OSError, ValueError):
        return None


def device_pci(dev):
    import torch
    pr = torch.cuda.get_device_properties(dev)
    return f"{pr.pci_domain_id:04x}:{pr.pci_bus_id:02x}:{pr.pci_device_id:02x}.0"


def require_distinct_devices(dev, world, rank):
    """A measured (non-rehearsal) N-rank run must have its N ranks on N distinct devices over RCCL:
    every rank's PCI address is gathered before any leg runs, and a world that does not satisfy it
    exits 4 on every rank without a line (a rehearsal says so with --rehearse)."""
    import torch.distributed as dist
    pcis = [None] * world
    dist.all_gather_object(pcis, device_pci(dev))
    backend = dist.get_backend()
    if backend == "nccl" and len(set(pcis)) == world:
        return
    if rank == 0:
        print(f"bench.py: {world} ranks on {len(set(pcis))} distinct device(s) {sorted(set(pcis))} over {backend}: "
              f"a measured N-rank run needs N distinct GPUs over RCCL ('nccl'); --rehearse for a one-GPU rehearsal",
              file=sys.stderr)
    dist.destroy_process_group()
    sys.exit(4)


def rank_info(dev, oks_batches):
    """This rank's identity and its headline result: device, PCI address, verdict digest of its
    own (rank-seeded, distinct) batches."""
    import torch
    pr = torch.cuda.get_device_properties(dev)
    ok = torch.cat([o.flatten() for o in oks_batches]).cpu().numpy()
    return {"rank": int(os.environ.get("RANK", "0")), "local_rank": int(os.environ.get("LOCAL_RANK", "0")),
            "device": str(dev), "name": pr.name, "pci": device_pci(dev),
            "uuid": str(getattr(pr, "uuid", "")), "verdicts_sha256": hashlib.sha256(ok.tobytes()).hexdigest()[:16],
            "passes": int(ok.sum()), "proofs": int(ok.size)}


def main():
    args = parse()
    rc = rank_launch(args)
    if rc is not None:
        sys.exit(rc)
    import torch
    import torch.distributed as dist

    import cudabulletproof_amd as bp
    from cudabulletproof_amd import synth

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # CPU baseline first, before this process touches the GPU: its worker processes are started
    # from a process with no HIP state (no fork/exec of a GPU-initialised process)
    # (at N > 1 the torchrun parent ran them before the spawn and hands them to rank 0)
    cpu, configs0, sample, launcher = None, None, None, None
    handed = cpu_legs_handed_over() if rank == 0 and world > 1 else None
    if handed is not None:
        cpu, configs0, launcher = handed["cpu_baseline"], handed["configs0"], handed["launcher"]
    elif not args.no_cpu and rank == 0:   # N = 1, or ranks started by an outer launcher (the driver's
        # torchrun): rank 0 runs them before init_process_group, the other ranks wait at the rendezvous
        cpu = cpu_baseline(args.n, args.cpu_seconds, args.cpu_procs)
        configs0 = configs0_leg()
    if rank == 0 and args.proofs == "prover" and not args.no_check:
        sample = oracle_sample(args.n, args.batch, seed=1)   # batch 0 of rank 0 (seed 1 + 1000 rank + 0)
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
    if world > 1 and not args.rehearse:
        require_distinct_devices(dev, world, rank)
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
    check = None
    if pipes and rank == 0 and not args.no_check:
        check = headline_check(B, n, pipes, streams, batches[0], Gd, Hd, hd, sample)

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
    # SURVEY 8(d) timing rule (>= 5 repetitions, median): the same K-step region 5 more times, the
    # pipelines still full; `value` stays the first region (the driver's contract), these go beside it
    reps = []
    for _ in range(0 if args.no_repeats else 5):
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize(dev)
        tr = time.perf_counter()
        for k in range(args.steps):
            step(k)
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()
        reps.append(time.perf_counter() - tr)
    for pp in pipes:
        pp.flush()
    torch.cuda.synchronize(dev)
    prefix_legs = None
    if pipes and args.table_legs.strip():   # the same workload at other table widths, e.g. none (K = 0)
        ref_oks = [o.clone() for o in oks[:nb]]
        prefix_legs = {f"k{b}": prefix_leg(args, dev, world, b, batches, ref_oks, Gd, Hd, gd, hd, streams)
                       for b in (int(x) for x in args.table_legs.split(",")) if b != args.prefix_bits}
    # every rank's identity + the verdicts of its own batches (gathered: proves N distinct ranks ran)
    ranks = [rank_info(dev, oks[:nb])]
    world_seen = 1
    if world > 1:
        world_seen = dist.get_world_size()
        ranks = [None] * world_seen
        dist.all_gather_object(ranks, rank_info(dev, oks[:nb]))
    h2d = None
    if pipes and not args.no_h2d:
        h2d = h2d_leg(args, dev, pipes, batches, args.steps, want_oks=oks[:nb] if args.mode == "pipeline" else None)
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
        if reps:
            t = torch.tensor(reps, dtype=torch.float64, device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            reps = [float(x) for x in t.tolist()]

    total = B * args.steps * world
    value = total / dt

    # dominant kernel + live roofline (HIP events on the verify stream)
    kern_ms = {k: v[0] for k, v in stats.items() if v[1]}
    dom = max(kern_ms, key=kern_ms.get)
    launches = stats[dom][1]
    avg_ms = stats[dom][0] / launches
    pcfg = {"batch_per_gpu": B, "n": n, "prefix_bits": prefix["bits"] if prefix else 0,
            "pipelines": len(pipes) or None}
    roofline, valu_roofline = rooflines(dom, B, n, args.steps, launches, avg_ms, dt, kern_ms, pcfg, len(pipes))
    roofline["scalar_mults_per_s"] = value * sm_per_verify(n)

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
            "n_gpus": world, "world_size": world_seen, "distinct_devices": len({r["pci"] for r in ranks}),
            "backend": dist.get_backend() if world > 1 else None, "ranks": ranks,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": dt / args.steps * 1e3,
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
                       "prefix_tables": prefix, "prefix_bits": prefix["bits"] if prefix else 0,
                       "prefix_tables_GB": round(prefix["GB"], 3) if prefix else 0.0,
                       "proof_bytes": proof_bytes(n, 1), "passes_in_warmup_batch": passes_warm},
            "prefix_legs": prefix_legs,
            "repeats": ({"n": len(reps), "steps_each": args.steps,
                         "median": total / statistics.median(reps), "min": total / max(reps),
                         "max": total / min(reps), "unit": "verifies/s",
                         "note": "the same K-step region 5 more times after `value`'s, pipelines full"}
                        if reps else None),
            "roofline": roofline, "valu_roofline": valu_roofline, "cpu_baseline": cpu, "verify_check": check,
            "with_h2d": h2d, "configs0": configs0, "msm": msm, "ipa": ipa, "prove": prove,
            "sharded_2p16": sharded, "host_api": host_api, "launcher": launcher,
        }
        for k, leg in (prefix_legs or {}).items():   # scalars in `config` (the driver keeps config's scalars)
            line["config"][f"{k}_value"] = leg["value"]
            line["config"][f"{k}_ms_per_step"] = leg["ms_per_step"]
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()   # the other ranks wait out rank 0's single-GPU legs, then all leave together
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
