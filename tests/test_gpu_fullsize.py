"""Parity at BASELINE.json's full sizes (configs[2] and configs[4]), where the oracle cannot run
the whole job inside a test:

* configs[2]: the 2^20-point canonical-tree MSM on SURVEY §8(d)'s config-3 inputs against the
  digest the CPU restatement produced (tests/golden/msm_2p20.json, make_msm_2p20.py), plus the
  size-independent decomposition property (per-shard roots == the oracle's shard roots, and
  the tree over them == the whole MSM).
* configs[4]: a 2^16-proof batch = 1024 distinct 64-bit proofs tiled x64 (SURVEY §8(d) config 5:
  the kernel must not dedupe) in ONE batched call: every tile returns exactly tile 0's verdicts,
  P and check points, and a sample of tile 0 matches the oracle.
"""
import hashlib
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN

pytestmark = pytest.mark.gpu


def d8(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()[:16]


def _msm_inputs(oracle, n):
    P = oracle.base_points(n, 5)
    s = np.stack([np.frombuffer(hashlib.sha256(b"msm-s" + i.to_bytes(4, "little")).digest(), "<u8")
                  for i in range(n)]).astype(np.uint64)
    s[:, 3] &= np.uint64(0x7FFFFFFFFFFFFFFF)
    return s, P


def test_msm_2p20_matches_oracle_digest(bp, oracle):
    import torch
    with open(os.path.join(GOLDEN, "msm_2p20.json")) as f:
        gold = json.load(f)
    n = gold["n"]
    s, P = _msm_inputs(oracle, n)
    dev = torch.device("cuda:0")
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a, np.uint64).view(np.int64)).to(dev)
    sd, Pd = T(s), T(P)
    out = torch.zeros(16, dtype=torch.int64, device=dev)
    bp.msm(out, sd, Pd)
    torch.cuda.synchronize()
    res = out.cpu().numpy().view(np.uint64)
    assert d8(res) == gold["digest"]
    assert [int(x) for x in res] == gold["result"]
    # decomposition: each aligned 2^17 shard's MSM is the oracle's shard root, and the canonical
    # tree over the roots (hipbp_point_tree) is the whole MSM again
    m = 1 << gold["shard_log2"]
    roots = torch.zeros(n // m, 16, dtype=torch.int64, device=dev)
    for k in range(n // m):
        bp.msm(roots[k], sd[k * m:(k + 1) * m], Pd[k * m:(k + 1) * m])
    torch.cuda.synchronize()
    assert np.array_equal(roots.cpu().numpy().view(np.uint64), np.array(gold["shard_roots"], np.uint64))
    top = torch.zeros(16, dtype=torch.int64, device=dev)
    bp.point_tree(top, roots)
    torch.cuda.synchronize()
    assert np.array_equal(top.cpu().numpy().view(np.uint64), res)


def test_batch_2p16_tiled_verify(bp, oracle):
    import torch
    from cudabulletproof_amd import synth
    n, distinct, tiles = 64, 1024, 64
    base = synth.proofs(distinct, n, seed=4242)
    base["c"][7] = base["c"][7] ^ np.uint64(1)        # a few failing proofs ride along
    base["t"][11] = 0
    arrays = {k: np.ascontiguousarray(np.concatenate([v] * tiles)) for k, v in base.items()}
    B = distinct * tiles
    G, H = oracle.base_points(n, 1), oracle.base_points(n, 2)
    g, h = oracle.gh()
    dev = torch.device("cuda:0")
    batch = bp.RangeProofBatch.from_numpy(n, arrays, dev)
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a, np.uint64).view(np.int64)).to(dev)
    ok = torch.zeros(B, dtype=torch.uint8, device=dev)
    P = torch.zeros(B, 16, dtype=torch.int64, device=dev)
    chk = torch.zeros(B, 16, dtype=torch.int64, device=dev)
    bp.batch_range_proof_verify(batch, T(G), T(H), T(g), T(h), ok, P, chk)
    torch.cuda.synchronize()
    ok = ok.cpu().numpy().astype(bool).reshape(tiles, distinct)
    P = P.cpu().numpy().view(np.uint64).reshape(tiles, distinct, 16)
    chk = chk.cpu().numpy().view(np.uint64).reshape(tiles, distinct, 16)
    assert (ok == ok[0]).all() and (P == P[0]).all() and (chk == chk[0]).all()
    assert not ok[0, 7]
    # every one of the 1024 distinct proofs against the CPU restatement (worker processes on the host)
    from oracle import pyoracle
    heads = np.stack([np.concatenate([base[k][p] for k in ("V", "A", "S", "T1", "T2")] +
                                     [np.zeros(8, np.uint64), base["t"][p], base["c"][p], base["x"][p]])
                      for p in range(distinct)])
    okr, Pr, chkr = pyoracle.cuda_range_proof_verify_many(n, heads, base["V"], base["a"], base["b"], base["L"],
                                                          base["R"], G, H, g, h)
    assert np.array_equal(ok[0], okr), np.nonzero(ok[0] != okr)[0][:10]
    assert np.array_equal(P[0], Pr)
    folds = okr | ~np.isin(np.arange(distinct), [7])   # every proof but the <a,b> != c one folds
    assert np.array_equal(chk[0][folds], chkr[folds])


def _proof_dicts(out, B):
    """Per-proof dicts (head, V, a, b, L, R as the reference harness lays them out) from the GPU
    prover's output tensors."""
    o = {k: out[k].cpu().numpy().view(np.uint64) for k in ("V", "A", "S", "T1", "T2", "taux", "mu", "t", "c", "x",
                                                          "a", "b", "L", "R")}
    return [dict(head=np.concatenate([o[k][p] for k in ("V", "A", "S", "T1", "T2", "taux", "mu", "t", "c", "x")]),
                 V=o["V"][p], a=o["a"][p], b=o["b"][p], L=o["L"][p], R=o["R"][p]) for p in range(B)]


@pytest.mark.parametrize("split", [False, True])
def test_batch1024_reference_outcomes(bp, oracle, golden, split):
    """BASELINE configs[1] at its full batch against the REFERENCE's own outcomes
    (tests/golden/batch1024.npz, make_golden.py make_batch1024): the GPU prover regenerates the
    1024 reference proofs (seeds + values; each proof's digest must equal the reference prover's,
    rp.cu:1159), and they go through the bench's exact configuration — ONE B = 1024 batch on one of
    two pipelines on their own streams, the bench's default prefix-table width, split stage 0 off
    and on — beside a second B = 1024 batch on the other pipeline whose first 256 proofs are the
    fixture's tampered copies.  Every verdict and every P digest, and the check-point digest of
    every case that folds, equal the reference's cuda_range_proof_verify (crv:82-127)."""
    import torch
    import bench
    from test_gpu_parity import _prove_inputs
    from test_accept_rule import _batch_arrays
    from accept_cases import apply_tamper
    d = golden("batch1024")
    n, B = 64, 1024
    dev = torch.device("cuda:0")
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a, np.uint64).view(np.int64)).to(dev)
    seeds = [int(d["seed0"]) + i for i in range(B)]
    values = [np.concatenate([np.frombuffer(np.uint64(x).tobytes(), np.uint8), np.zeros(24, np.uint8)])
              for x in d["value"]]
    v, gam, sL, sR, rnd, _ = _prove_inputs(seeds, values, n)
    G, H = oracle.base_points(n, 1), oracle.base_points(n, 2)
    g, h = oracle.gh()
    K = bench.DEFAULT_PREFIX_BITS
    gens = bp.Generators(n, T(G), T(H), T(g), T(h), prefix_bits=K)
    pipes = []
    try:
        out = bp.batch_generate_range_proof(n, T(v), T(gam), T(sL), T(sR), T(rnd), T(G), T(H), T(g), T(h), gens=gens)
        torch.cuda.synchronize()
        assert int(out["valid"].sum().item()) == B
        proofs = _proof_dicts(out, B)
        got = np.stack([np.frombuffer(hashlib.sha256(b"".join(np.ascontiguousarray(pr[k], np.uint64).tobytes()
                                                              for k in ("head", "V", "a", "b", "L", "R"))).digest()[:8],
                                      np.uint8) for pr in proofs])
        assert np.array_equal(got, d["proof_d8"]), "GPU prover != reference prover"
        batch0 = bp.RangeProofBatch(n, **{k: out[k] for k in bp.RangeProofBatch.FIELDS})
        tcases = [apply_tamper(proofs[int(b)], f, w, m) for (b, f, w), m in zip(d["tamper"], d["tamper_mask"])]
        batch1 = bp.RangeProofBatch.from_numpy(n, _batch_arrays(tcases + proofs[256:]), dev)
        streams = [torch.cuda.Stream(dev) for _ in range(2)]
        pipes = [bp.VerifyPipeline(B, n, T(G), T(H), T(h), stream=st) for st in streams]
        res = []
        for pp, b in zip(pipes, (batch0, batch1)):
            pp.use_gens(gens)
            pp.defer_msm(split)
            ok = torch.zeros(B, dtype=torch.uint8, device=dev)
            P = torch.zeros(B, 16, dtype=torch.int64, device=dev)
            chk = torch.zeros(B, 16, dtype=torch.int64, device=dev)
            pp.push(b, ok, P, chk)
            res.append((ok, P, chk))
        for pp in pipes:
            pp.flush()
        torch.cuda.synchronize()
    finally:
        for pp in pipes:
            pp.close()
        gens.close()
        torch.cuda.empty_cache()
    p8 = lambda P: np.stack([np.frombuffer(hashlib.sha256(r.tobytes()).digest()[:8], np.uint8)
                             for r in P.cpu().numpy().view(np.uint64)])
    want = [(d["ok"], d["P_d8"], d["check_d8"], d["early"]),
            (np.concatenate([d["t_ok"], d["ok"][256:]]), np.concatenate([d["t_P_d8"], d["P_d8"][256:]]),
             np.concatenate([d["t_check_d8"], d["check_d8"][256:]]), np.concatenate([d["t_early"], d["early"][256:]]))]
    for k, ((ok, P, chk), (wok, wP, wchk, wearly)) in enumerate(zip(res, want)):
        okh = ok.cpu().numpy().astype(bool)
        assert np.array_equal(okh, wok.astype(bool)), (k, np.nonzero(okh != wok.astype(bool))[0][:10])
        assert np.array_equal(p8(P), wP), k
        folds = ~wearly.astype(bool)
        assert np.array_equal(p8(chk)[folds], wchk[folds]), k
    assert 0 < int(d["ok"].sum()) <= B and int(d["t_ok"].sum()) < 256


def test_msm_pippenger_2p20_matches_oracle(bp, oracle):
    """hipbp_msm_pippenger (window 12, the labelled alternative) on the same 2^20 inputs equals
    orc_msm_pippenger's result (tests/golden/msm_2p20.json)."""
    import torch
    with open(os.path.join(GOLDEN, "msm_2p20.json")) as f:
        gold = json.load(f)
    s, P = _msm_inputs(oracle, gold["n"])
    dev = torch.device("cuda:0")
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a, np.uint64).view(np.int64)).to(dev)
    out = torch.zeros(16, dtype=torch.int64, device=dev)
    bp.msm_pippenger(out, T(s), T(P), 12)
    torch.cuda.synchronize()
    assert [int(x) for x in out.cpu().numpy().view(np.uint64)] == gold["pippenger_w12"]["result"]
