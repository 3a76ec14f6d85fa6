"""The tolerant accept rule of cuda_inner_product_verify (crv:287-367, nb:6816-6895) and the check
point it compares, pinned by what the REFERENCE PRINTS (tests/golden/make_golden.py `printed` and
`accept`, from oracle/_ref/libbpref.so with its stdout captured, oracle/ref/ref_harness.cc):

* "Computed X" (the first 8 bytes of tobytes(check.X)), "Expected X" (of P.X), the X / Y
  differing-byte and small-difference counts, "Matching significant bits" and "Hash difference
  count" of every case, and the early "<a,b> != c" reject (crv:146-158);
* `check_pin`: the reference's report when the same inner-product proof is verified against
  P := the fixture's check point.  0 differing bytes in X and Y means the composed check point
  (ref_ipa_fold) has exactly the reference's own X / Y bytes.

CPU tests: the fixtures are self-consistent with pyoracle.accept_stats (a restatement of crv:297-357),
every branch of the rule is reached, and the C restatement (oracle/bp_oracle.c) reproduces every
verdict, P and check point.  GPU test: the verify pipeline (lanes / pairs / quads forced, prefix
tables off and at the bench's K = 22) and cuda_inner_product_verify reproduce them too.
"""
import os
import sys

import numpy as np
import pytest

from oracle import pyoracle as po

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "golden"))
from accept_cases import accept_cases  # noqa: E402


def _xy(oracle, p):
    return np.concatenate([oracle.fe_tobytes(p[0:4]), oracle.fe_tobytes(p[4:8])]).tobytes()


def _stats_row(st):
    return [st[k] for k in po.STATS]


def _check_printed(oracle, check, P, x8c, x8e, stats):
    """The reference's printed figures == the figures recomputed from (check, P)."""
    cxy, pxy = _xy(oracle, check), _xy(oracle, P)
    assert bytes(x8c) == cxy[:8] and bytes(x8e) == pxy[:8]
    st = po.accept_stats(cxy, pxy)
    assert _stats_row(st) == list(stats)
    return st


def _pin_ok(pin):
    # X and Y identical: no differing byte, all 64 significant bits match (the hash count varies)
    return list(pin[:5]) == [0, 0, 0, 0, 64]


@pytest.mark.parametrize("n", [16, 64])
def test_reference_printed_check_points(oracle, golden, n):
    """proofs_n16/n64: the 6 reference proofs' check points and verdicts equal what the reference
    printed about them, and the reference itself reports 0 differing bytes against each stored
    check point (so the fixture's check point is reference-emitted, not only composed)."""
    d = golden(f"proofs_n{n}")
    assert not d["printed_early"].any()
    for i in range(len(d["head"])):
        st = _check_printed(oracle, d["check"][i], d["P"][i], d["printed_x8c"][i], d["printed_x8e"][i],
                            d["printed_stats"][i])
        assert st["verdict"] == bool(d["printed_ok"][i]) == bool(d["ok_cuda"][i])
        assert _pin_ok(d["check_pin"][i]), d["check_pin"][i]


def test_reference_printed_ipa4096(oracle, golden):
    d = golden("ipa4096")
    st = _check_printed(oracle, d["check"], d["P"], d["printed_x8c"], d["printed_x8e"], d["printed_stats"])
    assert st["verdict"] == bool(d["printed_ok"]) == bool(d["ok"])
    assert d["printed_early_raw"] == 1 and not d["printed_ok_raw"] and not d["ok_raw"]
    assert _pin_ok(d["printed_stats_pin"]) and d["printed_ok_pin"]


def _branches(stats):
    st = dict(zip(po.STATS, (int(x) for x in stats)))
    return {"b_small": st["small_x"] + st["small_y"] >= 20, "b_msb": st["msb"] >= 28,
            "b_diffs": st["x_diffs"] + st["y_diffs"] <= 32, "b_hash": st["hash_nonzero"] <= 24}


@pytest.mark.parametrize("n", [16, 64])
def test_accept_fixture_consistent_and_branches(oracle, golden, n):
    """accept_n*: every printed figure follows from the stored (check, P); every check point is
    pinned by the reference's zero-difference report; and every branch of the rule is reached by
    reference-emitted verdicts — the early reject, an accept decided by each of the small-count,
    significant-bits and differing-byte tests ALONE, and rejects with every test false.  The hash
    test (<= 24 non-zero bytes in a SHA-256 output) never holds: no input reaches it (~1e-12)."""
    d = golden(f"accept_n{n}")
    cases = accept_cases(d)
    assert len(cases) == len(d["ok"]) == 256
    alone = {b: 0 for b in po.BRANCHES}
    rejects_all_false = 0
    for i in range(len(cases)):
        if d["early"][i]:
            assert not d["ok"][i] and (d["stats"][i] == -1).all()
            continue
        st = _check_printed(oracle, d["check"][i], d["P"][i], d["x8c"][i], d["x8e"][i], d["stats"][i])
        assert st["verdict"] == bool(d["ok"][i])
        assert _pin_ok(d["check_pin"][i])
        br = _branches(d["stats"][i])
        if sum(br.values()) == 1:
            alone[[k for k, v in br.items() if v][0]] += 1
        rejects_all_false += not any(br.values())
    for i in range(len(d["ipa_ok"])):
        br = _branches(d["ipa_stats"][i])
        assert any(br.values()) == bool(d["ipa_ok"][i])
        if sum(br.values()) == 1:
            alone[[k for k, v in br.items() if v][0]] += 1
        rejects_all_false += not any(br.values())
    assert d["early"].sum() >= 20 and rejects_all_false >= 8
    assert alone["b_msb"] >= 10 and alone["b_small"] >= 8 and alone["b_diffs"] >= 8, alone
    assert alone["b_hash"] == 0
    assert not any(_branches(s)["b_hash"] for s in d["stats"] if s[0] >= 0)
    # the crafted variants decide as designed: 0 equal, 1 small count alone, 2 byte count alone, 3 none
    for i, v in enumerate(d["ipa_variant"]):
        br = _branches(d["ipa_stats"][i])
        want = [{"b_msb", "b_diffs"}, {"b_small"}, {"b_diffs"}, set()][int(v)]
        assert {k for k, x in br.items() if x} == want


@pytest.mark.parametrize("n", [16, 64])
def test_oracle_matches_reference_accept_cases(oracle, golden, n):
    """The C restatement on all 256 range-mode cases: verdict and P of every case, the check point
    of every case that folds; and the 32 crafted inner-product cases' verdicts."""
    d = golden(f"accept_n{n}")
    G, H, g, h = d["G"], d["H"], d["g"], d["h"]
    for i, pr in enumerate(accept_cases(d)):
        ok, P, chk, _, _ = oracle.cuda_range_proof_verify(pr["head"], pr["V"], n, pr["a"], pr["b"], pr["L"], pr["R"],
                                                         G, H, g, h)
        assert ok == bool(d["ok"][i]), i
        assert np.array_equal(P, d["P"][i]), i
        if not d["early"][i]:
            assert np.array_equal(chk, d["check"][i]), i
    for i in range(len(d["ipa_ok"])):
        b = int(d["ipa_base"][i])
        hd = po.head_fields(d["base_head"][b])
        ok, chk, _, _ = oracle.cuda_inner_product_verify(n, d["base_a"][b], d["base_b"][b], hd["c"], d["base_L"][b],
                                                         d["base_R"][b], hd["x"], d["ipa_P"][i], G, H, h)
        assert ok == bool(d["ipa_ok"][i]) and np.array_equal(chk, d["check"][b])


def _batch_arrays(cases):
    A = {k: [] for k in ("V", "A", "S", "T1", "T2", "t", "a", "b", "c", "x", "L", "R")}
    for pr in cases:
        hd = po.head_fields(pr["head"])
        A["V"].append(pr["V"])
        for k in ("A", "S", "T1", "T2", "t", "c", "x"):
            A[k].append(hd[k])
        for k in ("a", "b", "L", "R"):
            A[k].append(pr[k])
    return {k: np.ascontiguousarray(np.stack(v), np.uint64) for k, v in A.items()}


@pytest.mark.gpu
@pytest.mark.parametrize("n", [16, 64])
def test_gpu_accept_cases(bp, oracle, golden, monkeypatch, n):
    """All 256 reference-emitted cases through the verify pipeline in one batch: lanes, quads,
    pairs and 16-lane rows forced on every tick and the default tick forms, without prefix tables and with the
    bench's K = 22 tables — every verdict and P, and the check point of every case that folds,
    equal the reference's.  The 32 crafted inner-product cases through the pipeline in
    inner-product mode (P given) and the four variants of one proof through the C ABI's
    cuda_inner_product_verify give the reference's verdicts."""
    import torch
    dev = torch.device("cuda:0")
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a, np.uint64).view(np.int64)).to(dev)
    d = golden(f"accept_n{n}")
    G, H, g, h = d["G"], d["H"], d["g"], d["h"]
    arrays = _batch_arrays(accept_cases(d))
    B = len(arrays["V"])
    folds = ~d["early"].astype(bool)
    K = 22
    gens = bp.Generators(n, T(G), T(H), T(g), T(h), prefix_bits=K)
    batch = bp.RangeProofBatch.from_numpy(n, arrays, dev)
    try:
        for tables in (False, True):
            for q in (None, "0", "1", "2", "3"):
                if q is None:
                    monkeypatch.delenv("HIPBP_QUAD", raising=False)
                else:
                    monkeypatch.setenv("HIPBP_QUAD", q)
                pipe = bp.VerifyPipeline(B, n, T(G), T(H), T(h))
                if tables:
                    pipe.use_gens(gens)
                ok = torch.zeros(B, dtype=torch.uint8, device=dev)
                P = torch.zeros(B, 16, dtype=torch.int64, device=dev)
                chk = torch.zeros(B, 16, dtype=torch.int64, device=dev)
                pipe.push(batch, ok, P, chk)
                pipe.flush()
                torch.cuda.synchronize()
                pipe.close()
                tag = f"tables={tables} HIPBP_QUAD={q}"
                assert np.array_equal(ok.cpu().numpy().astype(bool), d["ok"].astype(bool)), tag
                assert np.array_equal(P.cpu().numpy().view(np.uint64), d["P"]), tag
                assert np.array_equal(chk.cpu().numpy().view(np.uint64)[folds], d["check"][folds]), tag
        monkeypatch.delenv("HIPBP_QUAD", raising=False)
        # crafted P, inner-product mode (cuda_inner_product_verify semantics, Q = h)
        base = accept_cases(d)[:24]
        ia = _batch_arrays([base[int(b)] for b in d["ipa_base"]])
        m = len(d["ipa_ok"])
        ib = bp.RangeProofBatch.from_numpy(n, ia, dev)
        pipe = bp.VerifyPipeline(m, n, T(G), T(H), T(h), range_mode=False)
        pipe.use_gens(gens)
        ok = torch.zeros(m, dtype=torch.uint8, device=dev)
        chk = torch.zeros(m, 16, dtype=torch.int64, device=dev)
        pipe.push(ib, ok, None, chk, P_in=T(d["ipa_P"]))
        pipe.flush()
        torch.cuda.synchronize()
        pipe.close()
        assert np.array_equal(ok.cpu().numpy().astype(bool), d["ipa_ok"].astype(bool))
        assert np.array_equal(chk.cpu().numpy().view(np.uint64), d["check"][d["ipa_base"]])
    finally:
        gens.close()
        torch.cuda.empty_cache()
    for i in range(4):   # the C ABI entry point, one proof per call
        b = int(d["ipa_base"][i])
        pr = base[b]
        assert bp.cuda_inner_product_verify(pr, d["ipa_P"][i], G, H, h) == bool(d["ipa_ok"][i])
