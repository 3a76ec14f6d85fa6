"""The CPU restatement (oracle/bp_oracle.c) against fixtures produced by the reference's own
code (tests/golden/make_golden.py) and against the survey's golden digests."""
import hashlib
import os

import numpy as np
import pytest

from conftest import GOLDEN


def d8(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()[:16]


def test_sha256_kats(oracle):
    # FIPS 180-4 examples
    assert oracle.sha256(b"abc").hex() == "ba7816bf8f01cfea414140de5dae2223b00361a396177a9cb410ff61f20015ad"
    assert oracle.sha256(b"").hex() == "e3b0c44298fc1c149afbf4c8996fb92427ae41e4649b934ca495991b7852b855"
    m = b"abcdbcdecdefdefgefghfghighijhijkijkljklmklmnlmnomnopnopq"
    assert oracle.sha256(m).hex() == "248d6a61d20638b8e5c026930c3e6039a33ce45964ff2167f6ecedd419db06c1"
    for n in (55, 56, 63, 64, 65, 119, 120, 200):
        data = bytes(range(256))[:n] * 1
        assert oracle.sha256(data) == hashlib.sha256(data).digest()


def test_field_against_reference(oracle, golden):
    d = golden("field")
    for i in range(len(d["f"])):
        f, g = d["f"][i], d["g"][i]
        assert np.array_equal(oracle.fe_add(f, g), d["add"][i]), i
        assert np.array_equal(oracle.fe_sub(f, g), d["sub"][i]), i
        assert np.array_equal(oracle.fe_mul(f, g), d["mul"][i]), i
        assert np.array_equal(oracle.fe_invert(f), d["invert"][i]), i
        assert np.array_equal(oracle.fe_tobytes(f), d["tobytes"][i]), i


def test_points_against_reference(oracle, golden):
    d = golden("point")
    for i in range(len(d["p"])):
        assert np.array_equal(oracle.ge_add(d["p"][i], d["q"][i]), d["add"][i]), i
        assert np.array_equal(oracle.ge_normalize_host(d["p"][i]), d["norm_host"][i]), i
        assert np.array_equal(oracle.ge_normalize_dev(d["p"][i]), d["norm_dev"][i]), i
    for i in range(len(d["scalars"])):
        assert np.array_equal(oracle.ge_scalarmult(d["scalars"][i], d["p"][i]), d["scalarmult"][i]), i


@pytest.mark.parametrize("n", [1, 2, 3, 5, 16, 17, 64])
def test_msm_against_reference(oracle, golden, n):
    d = golden("msm")
    assert np.array_equal(oracle.base_points(n, 5), d[f"P{n}"])
    assert np.array_equal(oracle.msm_canon(d[f"s{n}"], d[f"P{n}"]), d[f"canon{n}"])
    assert np.array_equal(oracle.msm_cpu(d[f"s{n}"], d[f"P{n}"]), d[f"cpu{n}"])


def test_survey_msm_digest(golden):
    # CanonTree MSM, points = base_points({5}), scalars = SHA256("msm-s"||i_le32) & bit255 cleared
    assert d8(golden("msm")["canon64"]) == "598ae9071d3bcf3a"


@pytest.mark.parametrize("n", [16, 64])
def test_verify_against_reference(oracle, golden, n):
    d = golden(f"proofs_n{n}")
    g2, h2 = oracle.gh()
    assert np.array_equal(g2, d["g"]) and np.array_equal(h2, d["h"])
    assert np.array_equal(oracle.base_points(n, 1), d["G"])
    for i in range(len(d["head"])):
        ok, P, chk, Gt, Ht = oracle.cuda_range_proof_verify(d["head"][i], d["V"][i], n, d["a"][i], d["b"][i], d["L"][i],
                                                            d["R"][i], d["G"], d["H"], d["g"], d["h"], trace=True)
        assert ok == bool(d["ok_cuda"][i]), i
        assert np.array_equal(P, d["P"][i]), i
        assert np.array_equal(chk, d["check"][i]), i
        assert np.array_equal(Gt, d["Gtrace"][i]) and np.array_equal(Ht, d["Htrace"][i]), i


def test_survey_proof_digests(golden):
    # SURVEY §8c golden digests (value = 42, seed 1)
    want = {16: ("96717c3978dc902a", "4567008fd60d9d07", "77bcc99376c5d8d0", "282f1a5824b8a457", "530e71ac9cbe3f9f"),
            64: ("96717c3978dc902a", "932119f12a0f5fa8", "8f64d8d9593c262b", "6df943dcd1bf5609", "ca6627284303a25d")}
    for n, (V, A, t, P, L) in want.items():
        d = golden(f"proofs_n{n}")
        head = d["head"][0]
        assert d8(d["V"][0]) == V
        assert d8(head[16:32]) == A
        assert d8(head[88:92]) == t
        assert d8(d["P"][0]) == P
        assert d8(d["L"][0]) == L


def test_ipa4096_against_reference(oracle, golden):
    """BASELINE configs[3]: the 4096-element inner-product argument (reference prover + verifier)."""
    import os
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "golden"))
    from make_golden import ipa_vectors
    d = golden("ipa4096")
    n = int(d["n"])
    G, H = oracle.base_points(n, 1), oracle.base_points(n, 2)
    _, Q = oracle.gh()
    a, b = ipa_vectors(n)
    assert np.array_equal(oracle.inner_product(a, b), d["c_in"])
    ok, chk, Gt, Ht = oracle.cuda_inner_product_verify(n, d["a"], d["b"], d["c_fix"], d["L"], d["R"], d["x"], d["P"],
                                                       G, H, Q, trace=True)
    assert ok == bool(d["ok"])
    assert np.array_equal(chk, d["check"])
    assert np.array_equal(Gt[-15:], d["Gtail"]) and np.array_equal(Ht[-15:], d["Htail"])
    ok_raw, _, _, _ = oracle.cuda_inner_product_verify(n, d["a"], d["b"], d["c_in"], d["L"], d["R"], d["x"], d["P"],
                                                       G, H, Q)
    assert ok_raw == bool(d["ok_raw"])


@pytest.mark.parametrize("n", [16, 64])
def test_range_proof_verify_against_reference(oracle, golden, n):
    """range_proof_verify (rp.cu:1717) — verdicts, delta and each sub-check."""
    d = golden("rpverify")
    G, H = oracle.base_points(n, 1), oracle.base_points(n, 2)
    g, h = oracle.gh()
    k = f"n{n}_"
    for i in range(len(d[k + "ok"])):
        ok, det = oracle.range_proof_verify(d[k + "head"][i], d[k + "V"][i], n, d[k + "a"][i], d[k + "b"][i],
                                            d[k + "L"][i], d[k + "R"][i], G, H, g, h)
        f = int(det["range_ok"]) | int(det["poly_ok"]) << 1 | int(det["ip_ok"]) << 2
        assert ok == bool(d[k + "ok"][i]), (i, d[k + "kind"][i])
        assert f == int(d[k + "flags"][i]), (i, d[k + "kind"][i])
        assert np.array_equal(det["delta"], d[k + "delta"][i]), i


def test_range_proof_verify_golden_proofs(oracle, golden):
    for n in (16, 64):
        d = golden(f"proofs_n{n}")
        for i in range(len(d["head"])):
            ok, _ = oracle.range_proof_verify(d["head"][i], d["V"][i], n, d["a"][i], d["b"][i], d["L"][i], d["R"][i],
                                              d["G"], d["H"], d["g"], d["h"])
            assert ok == bool(d["ok_cpu"][i]), (n, i)


@pytest.mark.parametrize("n", [16, 64])
def test_prover_against_reference(oracle, golden, n):
    """§8(f) rank 1: generate_range_proof + inner_product_prove + fix_inner_product_proof restated,
    on the reference's own proofs (same values, same RAND_bytes stream): every proof byte equal."""
    from oracle.pyoracle import prover_randomness
    d = golden(f"proofs_n{n}")
    for i in range(len(d["head"])):
        gamma, sLR, rnd4 = prover_randomness(i + 1, n)   # make_golden.py: seed = i + 1
        pr = oracle.generate_range_proof(d["value"][i], gamma, sLR, rnd4, n, d["G"], d["H"], d["g"], d["h"])
        assert np.array_equal(pr["head"], d["head"][i]), i
        for k in ("V", "a", "b", "L", "R"):
            assert np.array_equal(pr[k], d[k][i]), (i, k)


def test_oracle_batch1024_sample(oracle, golden):
    """batch1024.npz (BASELINE configs[1] at full batch, reference-emitted): a 24-case sample —
    every 64th of the 1024 reference proofs and every 32nd tampered copy — through the CPU
    restatement's prover and cuda_range_proof_verify: proof, P and check-point digests and the
    verdicts equal the reference's (the GPU runs the whole fixture: test_gpu_fullsize.py)."""
    import sys
    from oracle.pyoracle import prover_randomness
    sys.path.insert(0, GOLDEN)
    from accept_cases import apply_tamper
    d = golden("batch1024")
    n = 64
    G, H = oracle.base_points(n, 1), oracle.base_points(n, 2)
    g, h = oracle.gh()
    dig = lambda *arrs: np.frombuffer(hashlib.sha256(b"".join(np.ascontiguousarray(a, np.uint64).tobytes()
                                                              for a in arrs)).digest()[:8], np.uint8)

    def proof(i):
        val = np.zeros(32, np.uint8)
        val[:8] = np.frombuffer(np.uint64(d["value"][i]).tobytes(), np.uint8)
        gamma, sLR, rnd4 = prover_randomness(int(d["seed0"]) + i, n)
        return oracle.generate_range_proof(val, gamma, sLR, rnd4, n, G, H, g, h)

    def check(pr, ok_w, P_w, chk_w, early):
        ok, P, chk, _, _ = oracle.cuda_range_proof_verify(pr["head"], pr["V"], n, pr["a"], pr["b"], pr["L"], pr["R"],
                                                          G, H, g, h)
        assert ok == bool(ok_w) and np.array_equal(dig(P), P_w)
        if not early:
            assert np.array_equal(dig(chk), chk_w)
    for i in range(0, 1024, 64):
        pr = proof(i)
        assert np.array_equal(dig(*(pr[k] for k in ("head", "V", "a", "b", "L", "R"))), d["proof_d8"][i]), i
        check(pr, d["ok"][i], d["P_d8"][i], d["check_d8"][i], d["early"][i])
    for j in range(0, 256, 32):
        b, f, w = (int(x) for x in d["tamper"][j])
        pr = apply_tamper(proof(b), f, w, int(d["tamper_mask"][j]))
        assert np.array_equal(dig(*(pr[k] for k in ("head", "V", "a", "b", "L", "R"))), d["t_proof_d8"][j]), j
        check(pr, d["t_ok"][j], d["t_P_d8"][j], d["t_check_d8"][j], d["t_early"][j])


def test_prover_refuses_out_of_range(oracle):
    """validate_range_input (rp.cu:238): bit n or any higher byte set -> no proof."""
    from oracle.pyoracle import prover_randomness
    n = 16
    G, H = oracle.base_points(n, 1), oracle.base_points(n, 2)
    g, h = oracle.gh()
    gamma, sLR, rnd4 = prover_randomness(3, n)
    for bad in ((2, 0x01), (5, 0x80), (31, 0x01)):
        v = np.zeros(32, np.uint8)
        v[bad[0]] = bad[1]
        assert oracle.generate_range_proof(v, gamma, sLR, rnd4, n, G, H, g, h) is None
    v = np.zeros(32, np.uint8)
    v[0], v[1] = 0xFF, 0xFF                                # 2^16 - 1: in range
    assert oracle.generate_range_proof(v, gamma, sLR, rnd4, n, G, H, g, h) is not None


def test_msm_2p20_golden_consistent(oracle):
    """tests/golden/msm_2p20.json: the canonical tree over its 8 shard roots is its result."""
    import json
    with open(os.path.join(GOLDEN, "msm_2p20.json")) as f:
        gold = json.load(f)
    roots = np.array(gold["shard_roots"], np.uint64)
    assert roots.shape == (gold["n"] >> gold["shard_log2"], 16)
    assert [int(x) for x in oracle.point_tree(roots)] == gold["result"]


def test_pippenger_oracle_small_cases(oracle):
    """orc_msm_pippenger on tiny inputs against a direct Python statement of the same algorithm."""
    rng = np.random.default_rng(3)
    for n, c in ((1, 4), (5, 4), (9, 5)):
        P = oracle.base_points(n, 4)
        s = rng.integers(0, 2**64, size=(n, 4), dtype=np.uint64)
        s[0] = 0
        W, M = (256 + c - 1) // c, 16
        NB = 1 << c
        ident = np.zeros(16, np.uint64)
        ident[4] = ident[8] = 1
        add = oracle.ge_add

        def tree(L):
            L = list(L)
            st = 1
            while st < len(L):
                for i in range(0, len(L) - st, 2 * st):
                    L[i] = add(L[i], L[i + st])
                st *= 2
            return L[0]

        def digit(i, w):
            v = int(s[i, 0]) | int(s[i, 1]) << 64 | int(s[i, 2]) << 128 | int(s[i, 3]) << 192
            return (v >> (c * w)) & (NB - 1)
        Sw = []
        for w in range(W):
            B = [tree([P[i] for i in range(n) if digit(i, w) == b]) if any(digit(i, w) == b for i in range(n))
                 else ident for b in range(NB)]
            V = []
            for k in range(NB // M):
                R = S = B[k * M + M - 1]
                for j in range(M - 2, 0, -1):
                    R = add(R, B[k * M + j])
                    S = add(S, R)
                R = add(R, B[k * M])
                V.append(add(S, oracle.ge_scalarmult(np.frombuffer((k * M).to_bytes(32, "little"), np.uint8), R)))
            Sw.append(tree(V))
        T = Sw[-1]
        for w in range(W - 2, -1, -1):
            for _ in range(c):
                T = add(T, T)
            T = add(T, Sw[w])
        assert np.array_equal(oracle.msm_pippenger(s, P, c), T), (n, c)
