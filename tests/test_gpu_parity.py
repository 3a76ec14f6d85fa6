"""GPU parity: libcudabulletproof_hip.so (gfx950 kernels) against the reference's own outputs
(tests/golden/, produced by make_golden.py from the reference build) and against the CPU
restatement (oracle/) on seeded inputs.  Everything is bit-exact: this is integer arithmetic.
Run on the GPU box: python -m pytest tests -m gpu -q
"""
import hashlib
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def d8(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()[:16]


def rand_fe(rng, k, top=True):
    v = rng.integers(0, 2**64, size=(k, 4), dtype=np.uint64)
    if not top:
        v[:, 3] &= np.uint64(0x7FFFFFFFFFFFFFFF)
    return v


# ----------------------------------------------------------------------------- field ops
def test_field_ops_match_reference(bp, golden):
    d = golden("field")
    assert np.array_equal(bp.cuda_batch_field_add(d["f"], d["g"]), d["add"])
    assert np.array_equal(bp.cuda_batch_field_sub(d["f"], d["g"]), d["sub"])
    assert np.array_equal(bp.cuda_batch_field_mul(d["f"], d["g"]), d["mul"])
    assert np.array_equal(bp.cuda_batch_field_mul_karatsuba(d["f"], d["g"]), d["mul"])
    assert np.array_equal(bp.cuda_batch_field_invert(d["f"]), d["invert"])


def test_field_ops_random_vs_oracle(bp, oracle):
    rng = np.random.default_rng(7)
    f, g = rand_fe(rng, 4096), rand_fe(rng, 4096)
    add, sub, mul = bp.cuda_batch_field_add(f, g), bp.cuda_batch_field_sub(f, g), bp.cuda_batch_field_mul(f, g)
    sq = bp.cuda_batch_field_square(f)
    soa = bp.cuda_soa_field_add(f, g)
    for i in range(0, 4096, 7):
        assert np.array_equal(add[i], oracle.fe_add(f[i], g[i])), i
        assert np.array_equal(sub[i], oracle.fe_sub(f[i], g[i])), i
        assert np.array_equal(mul[i], oracle.fe_mul(f[i], g[i])), i
        assert np.array_equal(sq[i], oracle.fe_square_kernel(f[i])), i
    assert np.array_equal(soa, f + g)   # limbwise u64 add, wraps, no carry (cuda_field_ops.cu:521)


def test_field_ops_empty(bp):
    z = np.zeros((0, 4), np.uint64)
    assert bp.cuda_batch_field_add(z, z).shape == (0, 4)


# ----------------------------------------------------------------------------- MSM
@pytest.mark.parametrize("n", [1, 2, 3, 5, 16, 17, 64])
def test_msm_matches_reference(bp, golden, n):
    d = golden("msm")
    assert np.array_equal(bp.cuda_point_vector_multi_scalar_mul(d[f"s{n}"], d[f"P{n}"]), d[f"canon{n}"])


@pytest.mark.parametrize("n", [255, 256, 257, 700])
def test_msm_multiblock_vs_oracle(bp, oracle, n):
    rng = np.random.default_rng(n)
    P = oracle.base_points(n, 11)
    s = rand_fe(rng, n)
    s[::5] = 0                                   # zero scalars: 256 doublings of the identity
    s[1::7, 1:] = 0                              # short scalars: long leading-zero runs
    assert np.array_equal(bp.cuda_point_vector_multi_scalar_mul(s, P), oracle.msm_canon(s, P))


def test_msm_4096_survey_digest(bp, oracle):
    # n = 4096, points = base_points({5}), scalars = SHA256("msm-s"||i_le32), bit 255 cleared
    n = 4096
    P = oracle.base_points(n, 5)
    s = np.stack([np.frombuffer(hashlib.sha256(b"msm-s" + i.to_bytes(4, "little")).digest(), "<u8")
                  for i in range(n)]).astype(np.uint64)
    s[:, 3] &= np.uint64(0x7FFFFFFFFFFFFFFF)
    assert d8(bp.cuda_point_vector_multi_scalar_mul(s, P)) == "17b524ff179c621d"


@pytest.mark.parametrize("n", [1, 2, 3, 5, 16, 17, 64])
def test_msm_shared_matches_reference(bp, golden, n):
    """cuda_point_vector_multi_scalar_mul_shared (cuda_bulletproof.h:17): for n <= 64 the reference's
    shared-memory kernel defines the canonical tree (kernels.cu:141-168) — the golden results."""
    d = golden("msm")
    assert np.array_equal(bp.cuda_point_vector_multi_scalar_mul(d[f"s{n}"], d[f"P{n}"], shared=True), d[f"canon{n}"])


@pytest.mark.parametrize("n", [65, 257])
def test_msm_shared_large_n_vs_oracle(bp, oracle, n):
    """n > 64: the reference's _shared delegates to the standard path (kernels.cu:122-126)."""
    rng = np.random.default_rng(3 * n)
    P = oracle.base_points(n, 13)
    s = rand_fe(rng, n)
    s[::6] = 0
    want = oracle.msm_canon(s, P)
    assert np.array_equal(bp.cuda_point_vector_multi_scalar_mul(s, P, shared=True), want)
    assert np.array_equal(bp.cuda_point_vector_multi_scalar_mul(s, P), want)


def test_cuda_benchmark_hooks_run(bp, capfd):
    """The four cuda_benchmark_* hooks the reference declares (cuda_bulletproof.h:81-84) run on the
    GPU and print one line each; the range-proof one verifies real GPU-prover proofs through the
    reference's per-proof entry point and the batched host-struct one, whose verdicts must agree."""
    import ctypes
    L = bp.lib()
    L.cuda_benchmark_multi_scalar_mul(ctypes.c_int(2), ctypes.c_size_t(64))
    L.cuda_benchmark_inner_product(ctypes.c_int(2), ctypes.c_size_t(1000))
    L.cuda_benchmark_field_operations(ctypes.c_int(2), ctypes.c_size_t(4096))
    L.cuda_benchmark_range_proof(ctypes.c_int(8), ctypes.c_size_t(16))
    L.cuda_benchmark_range_proof(ctypes.c_int(4), ctypes.c_size_t(64))
    out = capfd.readouterr().out.splitlines()
    assert sum(l.startswith("cuda_benchmark_multi_scalar_mul: n=64") for l in out) == 1
    assert sum(l.startswith("cuda_benchmark_inner_product: n=1000") for l in out) == 1
    assert sum(l.startswith("cuda_benchmark_field_operations:") for l in out) == 3
    rp = [l for l in out if l.startswith("cuda_benchmark_range_proof:")]
    assert len(rp) == 2, out
    assert "n=16  8 proofs" in rp[0] and "verdicts agree 8/8" in rp[0], rp[0]
    assert "n=64  4 proofs" in rp[1] and "verdicts agree 4/4" in rp[1], rp[1]


def test_release_stream_workspaces(bp, oracle):
    """hipbp_release_stream_workspaces frees a stream's cached workspaces; the next call on that
    stream rebuilds them and gives the same bits (workspaces per short-lived stream)."""
    import torch
    dev = torch.device("cuda:0")
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a, np.uint64).view(np.int64)).to(dev)
    n = 3000
    rng = np.random.default_rng(77)
    P = oracle.base_points(n, 21)
    s = rand_fe(rng, n)
    want_p = oracle.msm_pippenger(s, P, 12)
    want_c = oracle.msm_canon(s[:300], P[:300])
    sd, Pd = T(s), T(P)
    for _ in range(3):
        st = torch.cuda.Stream(dev)
        out = torch.zeros(2, 16, dtype=torch.int64, device=dev)
        torch.cuda.synchronize()
        bp.msm_pippenger(out[0], sd, Pd, 12, stream=st)
        bp.msm(out[1], sd[:300], Pd[:300], stream=st)
        bp.release_stream_workspaces(st)   # waits for st first
        got = out.cpu().numpy().view(np.uint64)
        assert np.array_equal(got[0], want_p) and np.array_equal(got[1], want_c)
        del st
    bp.release_stream_workspaces(None)   # the null stream's workspaces (rebuilt by the next call on it)


def test_msm_length_mismatch_leaves_result(bp, capfd):
    import ctypes
    s = np.zeros((3, 4), np.uint64)
    P = np.zeros((2, 16), np.uint64)
    out = np.full(16, 7, np.uint64)
    sv = bp.FieldVector(s.ctypes.data, 3)
    pv = bp.PointVector(P.ctypes.data, 2)
    bp.lib().cuda_point_vector_multi_scalar_mul(ctypes.c_void_p(out.ctypes.data), ctypes.byref(sv), ctypes.byref(pv))
    assert (out == 7).all()
    assert "Vector lengths must match" in capfd.readouterr().err


# ----------------------------------------------------------------------------- inner products
@pytest.mark.parametrize("n", [1, 3, 16, 100, 512, 513, 4096, 70000])
def test_field_inner_product_orders(bp, oracle, n):
    rng = np.random.default_rng(n)
    a, b = rand_fe(rng, n), rand_fe(rng, n)
    assert np.array_equal(bp.cuda_field_vector_inner_product(a, b), oracle.ip_gpu(a, b))
    if n <= 1024:
        assert np.array_equal(bp.cuda_field_vector_inner_product(a, b, shared=True), oracle.ip_gpu(a, b, shared=True))


@pytest.mark.parametrize("n", [1, 64, 300])
def test_batch_field_inner_product(bp, oracle, n):
    rng = np.random.default_rng(3)
    a, b = rand_fe(rng, 5 * n).reshape(5, n, 4), rand_fe(rng, 5 * n).reshape(5, n, 4)
    assert np.array_equal(bp.cuda_batch_field_vector_inner_product(a, b), oracle.ip_gpu_batch(a, b))


# ----------------------------------------------------------------------------- verify
def _proof(d, i):
    return dict(head=d["head"][i], a=d["a"][i], b=d["b"][i], L=d["L"][i], R=d["R"][i])


@pytest.mark.parametrize("n", [16, 64])
def test_single_verify_matches_reference(bp, golden, n):
    d = golden(f"proofs_n{n}")
    for i in range(len(d["head"])):
        ok = bp.cuda_range_proof_verify(_proof(d, i), d["V"][i], n, d["G"], d["H"], d["g"], d["h"])
        assert ok == bool(d["ok_cuda"][i]), i
        ok2 = bp.cuda_inner_product_verify(_proof(d, i), d["P"][i], d["G"], d["H"], d["h"])
        assert ok2 == bool(d["ok_cuda"][i]), i


def test_single_verify_generator_reuse(bp, golden):
    """The single-proof calls keep the last generator set they uploaded and skip the copies when the
    next call brings the same bytes: alternating generator sets (G and H swapped), sizes (n = 16 / 64:
    the staging buffer grows) and the two entry points, every verdict equals the batch API's for the
    same proof and generators (which never reuses them)."""
    sets = {n: golden(f"proofs_n{n}") for n in (16, 64)}
    want = {}
    for n, d in sets.items():
        arrays = _batch_from_golden(bp, d, None)
        want[n, False] = _run_batch(bp, n, arrays, d["G"], d["H"], d["g"], d["h"])[0]
        want[n, True] = _run_batch(bp, n, arrays, d["H"], d["G"], d["g"], d["h"])[0]
    for rep in range(2):
        for n in (16, 64, 16):
            d = sets[n]
            for swap in (False, True, True, False):
                G, H = (d["H"], d["G"]) if swap else (d["G"], d["H"])
                for i in range(min(3, len(d["head"]))):
                    ok = bp.cuda_range_proof_verify(_proof(d, i), d["V"][i], n, G, H, d["g"], d["h"])
                    assert ok == bool(want[n, swap][i]), (rep, n, swap, i)
                    bp.cuda_inner_product_verify(_proof(d, i), d["P"][i], G, H, d["h"])


def _batch_from_golden(bp, d, device):
    from oracle.pyoracle import head_fields
    hs = [head_fields(h) for h in d["head"]]
    arrays = dict(V=d["V"], A=np.stack([h["A"] for h in hs]), S=np.stack([h["S"] for h in hs]),
                  T1=np.stack([h["T1"] for h in hs]), T2=np.stack([h["T2"] for h in hs]),
                  t=np.stack([h["t"] for h in hs]), a=d["a"], b=d["b"], c=np.stack([h["c"] for h in hs]),
                  x=np.stack([h["x"] for h in hs]), L=d["L"], R=d["R"])
    return arrays


def _run_batch(bp, n, arrays, G, H, g, h):
    import torch
    dev = torch.device("cuda:0")
    batch = bp.RangeProofBatch.from_numpy(n, arrays, dev)
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a, np.uint64).view(np.int64)).to(dev)
    B = batch.count
    ok = torch.zeros(B, dtype=torch.uint8, device=dev)
    P = torch.zeros(B, 16, dtype=torch.int64, device=dev)
    chk = torch.zeros(B, 16, dtype=torch.int64, device=dev)
    bp.batch_range_proof_verify(batch, T(G), T(H), T(g), T(h), ok, P, chk)
    torch.cuda.synchronize()
    return ok.cpu().numpy().astype(bool), P.cpu().numpy().view(np.uint64), chk.cpu().numpy().view(np.uint64)


@pytest.mark.parametrize("n", [16, 64])
def test_batch_verify_matches_reference(bp, golden, n):
    d = golden(f"proofs_n{n}")
    ok, P, chk = _run_batch(bp, n, _batch_from_golden(bp, d, None), d["G"], d["H"], d["g"], d["h"])
    assert np.array_equal(ok, d["ok_cuda"].astype(bool))
    assert np.array_equal(P, d["P"])
    assert np.array_equal(chk, d["check"])


def _synth_proof_dicts(s, n):
    out = []
    for i in range(len(s["V"])):
        head = np.concatenate([s[k][i] for k in ("V", "A", "S", "T1", "T2")] +
                              [np.zeros(8, np.uint64), s["t"][i], s["c"][i], s["x"][i]])
        out.append(dict(head=head, a=s["a"][i], b=s["b"][i], L=s["L"][i], R=s["R"][i]))
    return out


@pytest.mark.parametrize("n", [16, 64])
def test_batch_verify_host_structs(bp, golden, n):
    """hipbp_batch_range_proof_verify_host over arrays of the reference's RangeProof structs: the
    reference proofs give the reference's verdicts; 2500 synthetic proofs (two 2048-proof pipeline
    ticks) give the device batch API's verdicts; a proof whose ip.n != n fails the reference's
    length check; one with a different a/b length takes the single-proof path and agrees with it."""
    import torch
    from cudabulletproof_amd import synth
    d = golden(f"proofs_n{n}")
    ref = [_proof(d, i) for i in range(len(d["head"]))]
    s = synth.proofs(2500, n, seed=500 + n)
    syn = _synth_proof_dicts(s, n)
    dev = torch.device("cuda:0")
    batch = bp.RangeProofBatch.from_numpy(n, s, dev)
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a, np.uint64).view(np.int64)).to(dev)
    okd = torch.zeros(2500, dtype=torch.uint8, device=dev)
    bp.batch_range_proof_verify(batch, T(d["G"]), T(d["H"]), T(d["g"]), T(d["h"]), okd)
    torch.cuda.synchronize()
    want_syn = okd.cpu().numpy().astype(bool)
    # a different a/b length (3): the single-proof path
    odd = dict(syn[7])
    rng = np.random.default_rng(n)
    odd["a"] = rand_fe(rng, 3)
    odd["b"] = rand_fe(rng, 3)
    want_odd = bp.cuda_range_proof_verify(odd, s["V"][7], n, d["G"], d["H"], d["g"], d["h"])
    proofs = ref + syn[:1200] + [odd] + syn[1200:]
    V = np.concatenate([d["V"], s["V"][:1200], s["V"][7:8], s["V"][1200:]])
    want = np.concatenate([d["ok_cuda"].astype(bool), want_syn[:1200], [want_odd], want_syn[1200:]])
    for ng in (1, 0):
        got = bp.batch_range_proof_verify_host(proofs, V, n, d["G"], d["H"], d["g"], d["h"], num_gpus=ng)
        assert np.array_equal(got, want), (ng, np.nonzero(got != want)[0][:10])
    # the generators' prefix tables the host path caches across calls: the same verdicts without
    # tables (HIPBP_HOST_PREFIX_BITS=0) and at other widths, and after a call with another generator
    # set (G and H swapped: the cache is rebuilt for it, then for the original set again)
    def host(G, H, m, bits=None):
        if bits is not None:
            os.environ["HIPBP_HOST_PREFIX_BITS"] = bits
        try:
            return bp.batch_range_proof_verify_host(proofs[:m], V[:m], n, G, H, d["g"], d["h"])
        finally:
            os.environ.pop("HIPBP_HOST_PREFIX_BITS", None)
    swapped = host(d["H"], d["G"], 40, "0")   # no tables: the plain arithmetic's verdicts for (H, G)
    assert np.array_equal(host(d["H"], d["G"], 40), swapped)
    for bits in ("0", "8", None):
        got = host(d["G"], d["H"], len(proofs), bits)
        assert np.array_equal(got, want), (bits, np.nonzero(got != want)[0][:10])
    assert np.array_equal(host(d["H"], d["G"], 40), swapped)
    # the multi-device path (shards cut from the index list, one host thread each, verdicts merged),
    # here with every shard on this box's one GPU: 2 and 3 shards give the same verdicts
    for k in ("2", "3"):
        os.environ["HIPBP_HOST_SHARDS"] = k
        try:
            got = bp.batch_range_proof_verify_host(proofs, V, n, d["G"], d["H"], d["g"], d["h"])
        finally:
            del os.environ["HIPBP_HOST_SHARDS"]
        assert np.array_equal(got, want), (k, np.nonzero(got != want)[0][:10])
    # the reference's length check (crv:140-143): generator vectors shorter than the proofs' n
    got = bp.batch_range_proof_verify_host(ref[:2], d["V"][:2], n, d["G"][:n // 2], d["H"][:n // 2], d["g"], d["h"])
    assert not got.any()
    # more devices than are visible: an error with a message, not a silent one-device run
    ndev = torch.cuda.device_count()
    with pytest.raises(bp.BulletproofError, match=f"num_gpus = {ndev + 1} but {ndev} HIP device"):
        bp.batch_range_proof_verify_host(ref, d["V"], n, d["G"], d["H"], d["g"], d["h"], num_gpus=ndev + 1)


@pytest.mark.parametrize("n,B,ab_len", [(64, 48, 1), (16, 40, 3), (4, 17, 2), (1, 9, 1), (256, 4, 1), (512, 3, 1),
                                        (1024, 2, 2),
                                        # B >= 64: lanes in chain-length order (the pipeline's lane sort)
                                        (64, 72, 1), (16, 130, 2), (4, 64, 1), (1, 70, 1), (2, 65, 1),
                                        (128, 64, 1)])
def test_batch_verify_synthetic_vs_oracle(bp, oracle, n, B, ab_len):
    from cudabulletproof_amd import synth
    arrays = synth.proofs(B, n, seed=1000 + n)
    rng = np.random.default_rng(n + B)
    if ab_len > 1:
        arrays["a"] = rand_fe(rng, B * ab_len).reshape(B, ab_len, 4)
        arrays["b"] = rand_fe(rng, B * ab_len).reshape(B, ab_len, 4)
        for p in range(B):   # make <a,b> = c for most proofs, leave a few failing
            if p % 5:
                arrays["c"][p] = oracle.inner_product(arrays["a"][p], arrays["b"][p])
    arrays["c"][B - 1] = rand_fe(rng, 1)[0]      # a <a,b> != c proof (crv:153 early reject)
    arrays["t"][B // 2] = 0                     # t = 0: 256 doublings of the identity
    G, H = oracle.base_points(n, 1), oracle.base_points(n, 2)
    g, h = oracle.gh()
    ok, P, chk = _run_batch(bp, n, arrays, G, H, g, h)
    head_keys = ("V", "A", "S", "T1", "T2")
    for p in range(B):
        head = np.concatenate([arrays[k][p] for k in head_keys] +
                              [np.zeros(4, np.uint64), np.zeros(4, np.uint64), arrays["t"][p], arrays["c"][p],
                               arrays["x"][p]])
        okr, Pr, chkr, _, _ = oracle.cuda_range_proof_verify(head, arrays["V"][p], n, arrays["a"][p], arrays["b"][p],
                                                             arrays["L"][p], arrays["R"][p], G, H, g, h)
        assert ok[p] == okr, p
        assert np.array_equal(P[p], Pr), p
        if okr or not np.array_equal(chkr, np.zeros(16, np.uint64)):
            assert np.array_equal(chk[p], chkr), p


def test_batch_verify_deterministic(bp, oracle):
    from cudabulletproof_amd import synth
    n = 64
    arrays = synth.proofs(96, n, seed=5)
    G, H = oracle.base_points(n, 1), oracle.base_points(n, 2)
    g, h = oracle.gh()
    r1 = _run_batch(bp, n, arrays, G, H, g, h)
    r2 = _run_batch(bp, n, arrays, G, H, g, h)
    for x, y in zip(r1, r2):
        assert np.array_equal(x, y)


# ----------------------------------------------------------------------------- streaming pipeline
@pytest.mark.parametrize("n", [16, 64])
def test_pipeline_matches_reference(bp, golden, n):
    """Batches of different sizes in flight together (hipbp_pipeline_*): each batch's verdicts,
    P and check points equal the reference's, whatever shares its ticks."""
    import torch
    d = golden(f"proofs_n{n}")
    arrays = _batch_from_golden(bp, d, None)
    dev = torch.device("cuda:0")
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a, np.uint64).view(np.int64)).to(dev)
    pipe = bp.VerifyPipeline(8, n, T(d["G"]), T(d["H"]), T(d["h"]))
    splits = [(0, 2), (2, 3), (3, 6), (0, 6), (5, 6)]
    outs = []
    for lo, hi in splits:
        sub = {k: v[lo:hi] for k, v in arrays.items()}
        batch = bp.RangeProofBatch.from_numpy(n, sub, dev)
        ok = torch.zeros(hi - lo, dtype=torch.uint8, device=dev)
        P = torch.zeros(hi - lo, 16, dtype=torch.int64, device=dev)
        chk = torch.zeros(hi - lo, 16, dtype=torch.int64, device=dev)
        pipe.push(batch, ok, P, chk)
        outs.append((lo, hi, ok, P, chk, batch))
        pipe.push(None)                      # a drain tick in between
    pipe.flush()
    torch.cuda.synchronize()
    for lo, hi, ok, P, chk, _ in outs:
        assert np.array_equal(ok.cpu().numpy().astype(bool), d["ok_cuda"][lo:hi].astype(bool))
        assert np.array_equal(P.cpu().numpy().view(np.uint64), d["P"][lo:hi])
        assert np.array_equal(chk.cpu().numpy().view(np.uint64), d["check"][lo:hi])
    pipe.close()


def test_pipeline_inner_product_mode(bp, golden):
    """range_mode 0 (cuda_inner_product_verify semantics) with the reference's P given."""
    import torch
    n = 64
    d = golden(f"proofs_n{n}")
    arrays = _batch_from_golden(bp, d, None)
    dev = torch.device("cuda:0")
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a, np.uint64).view(np.int64)).to(dev)
    pipe = bp.VerifyPipeline(8, n, T(d["G"]), T(d["H"]), T(d["h"]), range_mode=False)
    batch = bp.RangeProofBatch.from_numpy(n, arrays, dev)
    ok = torch.zeros(batch.count, dtype=torch.uint8, device=dev)
    chk = torch.zeros(batch.count, 16, dtype=torch.int64, device=dev)
    pipe.push(batch, ok, None, chk, P_in=T(d["P"]))
    pipe.flush()
    torch.cuda.synchronize()
    assert np.array_equal(ok.cpu().numpy().astype(bool), d["ok_cuda"].astype(bool))
    assert np.array_equal(chk.cpu().numpy().view(np.uint64), d["check"])
    pipe.close()


# ----------------------------------------------------------------------------- IPA n = 4096 (configs[3])
def _ipa4096(golden, oracle):
    import os
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "golden"))
    from make_golden import ipa_vectors  # noqa: F401  (vectors only matter for P, which is recorded)
    d = golden("ipa4096")
    n = int(d["n"])
    G, H = oracle.base_points(n, 1), oracle.base_points(n, 2)
    _, Q = oracle.gh()
    return d, n, G, H, Q


def test_ipa4096_single_call_matches_reference(bp, golden, oracle):
    """cuda_inner_product_verify (C ABI, host buffers) at n = 4096."""
    d, n, G, H, Q = _ipa4096(golden, oracle)
    z = np.zeros(100, np.uint64)
    for c, want in ((d["c_fix"], d["ok"]), (d["c_in"], d["ok_raw"])):
        head = z.copy()
        head[92:96] = c
        head[96:100] = d["x"]
        proof = dict(head=head, a=d["a"], b=d["b"], L=d["L"], R=d["R"])
        assert bp.cuda_inner_product_verify(proof, d["P"], G, H, Q) == bool(want)


@pytest.mark.parametrize("B", [6, 66])   # 66: lanes in chain-length order (lane sort)
def test_ipa4096_batch_matches_reference(bp, golden, oracle, B):
    """hipbp_batch_inner_product_verify over a batch of 4096-element IPAs: verdicts and the
    check point equal the reference's; rejected-at-<a,b> proofs leave no check point."""
    import torch
    d, n, G, H, Q = _ipa4096(golden, oracle)
    dev = torch.device("cuda:0")
    zero_pt = np.zeros((B, 16), np.uint64)
    c = np.stack([d["c_fix"] if p % 3 else d["c_in"] for p in range(B)])
    arrays = dict(V=zero_pt, A=zero_pt, S=zero_pt, T1=zero_pt, T2=zero_pt, t=np.zeros((B, 4), np.uint64),
                  a=np.repeat(d["a"][None], B, 0), b=np.repeat(d["b"][None], B, 0), c=c,
                  x=np.repeat(d["x"][None], B, 0), L=np.repeat(d["L"][None], B, 0), R=np.repeat(d["R"][None], B, 0))
    batch = bp.RangeProofBatch.from_numpy(n, arrays, dev)
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a, np.uint64).view(np.int64)).to(dev)
    ok = torch.zeros(B, dtype=torch.uint8, device=dev)
    chk = torch.zeros(B, 16, dtype=torch.int64, device=dev)
    bp.batch_inner_product_verify(batch, T(np.repeat(d["P"][None], B, 0)), T(G), T(H), T(Q), ok, chk)
    torch.cuda.synchronize()
    ok = ok.cpu().numpy().astype(bool)
    chk = chk.cpu().numpy().view(np.uint64)
    for p in range(B):
        if p % 3:
            assert ok[p] == bool(d["ok"]) and np.array_equal(chk[p], d["check"]), p
        else:
            assert ok[p] == bool(d["ok_raw"]), p


# ----------------------------------------------------------------------------- range_proof_verify (A18)
def _std_arrays(heads, V, a, b, L, R):
    from oracle.pyoracle import head_fields
    hs = [head_fields(h) for h in heads]
    return dict(V=np.asarray(V), A=np.stack([h["A"] for h in hs]), S=np.stack([h["S"] for h in hs]),
                T1=np.stack([h["T1"] for h in hs]), T2=np.stack([h["T2"] for h in hs]),
                t=np.stack([h["t"] for h in hs]), a=np.asarray(a), b=np.asarray(b),
                c=np.stack([h["c"] for h in hs]), x=np.stack([h["x"] for h in hs]), L=np.asarray(L), R=np.asarray(R),
                taux=np.stack([h["taux"] for h in hs]), mu=np.stack([h["mu"] for h in hs]),
                Vp=np.stack([np.asarray(h_)[0:16] for h_ in heads]))


def _run_std(bp, n, arrays, G, H, g, h):
    import torch
    dev = torch.device("cuda:0")
    batch = bp.RangeProofBatch.from_numpy(n, arrays, dev)
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a, np.uint64).view(np.int64)).to(dev)
    B = batch.count
    ok = torch.zeros(B, dtype=torch.uint8, device=dev)
    P = torch.zeros(B, 16, dtype=torch.int64, device=dev)
    chk = torch.zeros(B, 16, dtype=torch.int64, device=dev)
    fl = torch.zeros(B, dtype=torch.uint8, device=dev)
    poly = torch.zeros(B, 4, 16, dtype=torch.int64, device=dev)
    bp.batch_range_proof_verify_std(batch, T(G), T(H), T(g), T(h), ok, P, chk, fl, poly)
    torch.cuda.synchronize()
    u = lambda t: t.cpu().numpy().view(np.uint64)
    return ok.cpu().numpy().astype(bool), u(P), u(chk), fl.cpu().numpy(), u(poly)


def _check_std_vs_oracle(oracle, n, arrays, heads, G, H, g, h, res, ref_ok=None, ref_flags=None):
    ok, P, chk, fl, poly = res
    for p in range(len(heads)):
        okr, det = oracle.range_proof_verify(heads[p], arrays["V"][p], n, arrays["a"][p], arrays["b"][p],
                                             arrays["L"][p], arrays["R"][p], G, H, g, h)
        assert ok[p] == okr, p
        if ref_ok is not None:
            assert ok[p] == bool(ref_ok[p]), p
        f = int(fl[p])
        assert bool(f & 1) == det["vmatch"] and bool(f & 2) == det["range_ok"], p
        assert bool(f & 4) == (det["poly_m1"] or det["poly_m2"]), p
        assert bool(f & 8) == det["poly_m3"] and bool(f & 16) == det["poly_m4"], p
        assert bool(f & 32) == det["ip_ok"], p
        if ref_flags is not None:
            rf = int(ref_flags[p])
            assert bool(rf & 1) == bool(f & 2) and bool(rf & 2) == bool(f & 28) and bool(rf & 4) == bool(f & 32), p
        assert np.array_equal(P[p], det["P"]), p
        for i, k in enumerate(("left", "right", "left_mult", "right_mult")):
            assert np.array_equal(poly[p, i], det[k]), (p, k)
        if det["ip_ok"] or not np.array_equal(det["check"], np.zeros(16, np.uint64)):
            assert np.array_equal(chk[p], det["check"]), p


@pytest.mark.parametrize("n", [16, 64])
def test_std_verify_matches_reference(bp, oracle, golden, n):
    """range_proof_verify semantics on the reference's proofs, tampered copies and random inputs:
    verdicts and sub-check results equal the reference's; every intermediate point equals the oracle's."""
    d = golden("rpverify")
    k = f"n{n}_"
    G, H = oracle.base_points(n, 1), oracle.base_points(n, 2)
    g, h = oracle.gh()
    heads = d[k + "head"]
    arrays = _std_arrays(heads, d[k + "V"], d[k + "a"], d[k + "b"], d[k + "L"], d[k + "R"])
    res = _run_std(bp, n, arrays, G, H, g, h)
    _check_std_vs_oracle(oracle, n, arrays, heads, G, H, g, h, res, d[k + "ok"], d[k + "flags"])


@pytest.mark.parametrize("n", [16, 64])
def test_std_verify_golden_proofs(bp, oracle, golden, n):
    d = golden(f"proofs_n{n}")
    heads = d["head"]
    arrays = _std_arrays(heads, d["V"], d["a"], d["b"], d["L"], d["R"])
    res = _run_std(bp, n, arrays, d["G"], d["H"], d["g"], d["h"])
    assert np.array_equal(res[0], d["ok_cpu"].astype(bool))
    _check_std_vs_oracle(oracle, n, arrays, heads, d["G"], d["H"], d["g"], d["h"], res)


@pytest.mark.parametrize("n,B,ab_len", [(64, 20, 1), (16, 9, 2), (1, 5, 1), (2, 3, 1), (256, 2, 1), (16, 70, 1),
                                        (64, 64, 1)])
def test_std_verify_synthetic_vs_oracle(bp, oracle, n, B, ab_len):
    from cudabulletproof_amd import synth
    arrays = synth.proofs(B, n, seed=500 + n)
    rng = np.random.default_rng(n)
    if ab_len > 1:
        arrays["a"] = rand_fe(rng, B * ab_len).reshape(B, ab_len, 4)
        arrays["b"] = rand_fe(rng, B * ab_len).reshape(B, ab_len, 4)
        for p in range(B - 1):
            arrays["c"][p] = oracle.inner_product(arrays["a"][p], arrays["b"][p])
    arrays["taux"] = rand_fe(rng, B, top=False)
    arrays["mu"] = rand_fe(rng, B, top=False)
    arrays["Vp"] = arrays["V"].copy()
    arrays["Vp"][0, 4] ^= np.uint64(1)            # V argument != proof V
    heads = np.concatenate([arrays[k] for k in ("Vp", "A", "S", "T1", "T2", "taux", "mu", "t", "c", "x")], axis=1)
    G, H = oracle.base_points(n, 1), oracle.base_points(n, 2)
    g, h = oracle.gh()
    res = _run_std(bp, n, arrays, G, H, g, h)
    assert not res[0][0]
    _check_std_vs_oracle(oracle, n, arrays, heads, G, H, g, h, res)


# ----------------------------------------------------------------------------- prover (§8(f) rank 1)
def _prove_inputs(seeds, values, n):
    from oracle.pyoracle import prover_randomness
    B = len(seeds)
    gam = np.zeros((B, 4), np.uint64)
    sL = np.zeros((B, n, 4), np.uint64)
    sR = np.zeros((B, n, 4), np.uint64)
    rnd = np.zeros((B, 4, 4), np.uint64)
    rb = []
    for p, sd in enumerate(seeds):
        gamma, sLR, rnd4 = prover_randomness(sd, n)
        gam[p] = gamma.view("<u8")
        sL[p] = sLR[:, :32].copy().view("<u8").reshape(n, 4)
        sR[p] = sLR[:, 32:].copy().view("<u8").reshape(n, 4)
        rnd[p] = rnd4.view("<u8").reshape(4, 4)
        rb.append((gamma, sLR, rnd4))
    v = np.stack([np.asarray(x, np.uint8).view("<u8") for x in values]).astype(np.uint64)
    return v, gam, sL, sR, rnd, rb


def _run_prover(bp, n, v, gam, sL, sR, rnd, G, H, g, h):
    import torch
    dev = torch.device("cuda:0")
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a, np.uint64).view(np.int64)).to(dev)
    out = bp.batch_generate_range_proof(n, T(v), T(gam), T(sL), T(sR), T(rnd), T(G), T(H), T(g), T(h))
    torch.cuda.synchronize()
    return {k: (t.cpu().numpy().view(np.uint64) if k != "valid" else t.cpu().numpy())
            for k, t in out.items() if k != "_keep"}


@pytest.mark.parametrize("n", [16, 64])
def test_prover_matches_reference(bp, golden, n):
    """The GPU prover reproduces the reference's own proofs byte for byte (same values, same RNG)."""
    d = golden(f"proofs_n{n}")
    B = len(d["head"])
    v, gam, sL, sR, rnd, _ = _prove_inputs(list(range(1, B + 1)), d["value"], n)
    o = _run_prover(bp, n, v, gam, sL, sR, rnd, d["G"], d["H"], d["g"], d["h"])
    from oracle.pyoracle import head_fields
    for p in range(B):
        hf = head_fields(d["head"][p])
        assert o["valid"][p] == 1
        for k in ("V", "A", "S", "T1", "T2", "taux", "mu", "t", "c", "x"):
            assert np.array_equal(o[k][p], hf[k]), (p, k)
        assert np.array_equal(o["V"][p], d["V"][p])
        assert np.array_equal(o["a"][p], d["a"][p]) and np.array_equal(o["b"][p], d["b"][p]), p
        assert np.array_equal(o["L"][p], d["L"][p]) and np.array_equal(o["R"][p], d["R"][p]), p


@pytest.mark.parametrize("n,B", [(1, 3), (2, 4), (8, 5), (32, 6), (128, 2)])
def test_prover_vs_oracle(bp, oracle, n, B):
    """Random values (some out of range: refused like the reference) vs the oracle's prover."""
    rng = np.random.default_rng(n * 7 + B)
    values = []
    for p in range(B):
        val = np.zeros(32, np.uint8)
        nb = max(1, n // 8)
        val[:nb] = rng.integers(0, 256, nb)
        if n % 8:
            val[0] &= (1 << n) - 1
        if p == B - 1:
            val[min(31, n // 8)] |= 1 << (n % 8)       # bit n set: refused (rp.cu:238)
        values.append(val)
    seeds = [1000 + 17 * p + n for p in range(B)]
    v, gam, sL, sR, rnd, rb = _prove_inputs(seeds, values, n)
    G, H = oracle.base_points(n, 1), oracle.base_points(n, 2)
    g, h = oracle.gh()
    o = _run_prover(bp, n, v, gam, sL, sR, rnd, G, H, g, h)
    for p in range(B):
        gamma, sLR, rnd4 = rb[p]
        pr = oracle.generate_range_proof(values[p], gamma, sLR, rnd4, n, G, H, g, h)
        if pr is None:
            assert o["valid"][p] == 0, p
            continue
        assert o["valid"][p] == 1, p
        from oracle.pyoracle import head_fields
        hf = head_fields(pr["head"])
        for k in ("V", "A", "S", "T1", "T2", "taux", "mu", "t", "c", "x"):
            assert np.array_equal(o[k][p], hf[k]), (p, k)
        assert np.array_equal(o["a"][p], pr["a"]) and np.array_equal(o["b"][p], pr["b"]), p
        assert np.array_equal(o["L"][p], pr["L"]) and np.array_equal(o["R"][p], pr["R"]), p


def test_prove_then_verify_on_gpu(bp, oracle):
    """Proofs made on the GPU verify on the GPU exactly as the reference's verifier judges them."""
    import torch
    n, B = 16, 12
    rng = np.random.default_rng(3)
    values = [np.concatenate([rng.integers(0, 256, 2).astype(np.uint8), np.zeros(30, np.uint8)]) for _ in range(B)]
    v, gam, sL, sR, rnd, _ = _prove_inputs([50 + p for p in range(B)], values, n)
    G, H = oracle.base_points(n, 1), oracle.base_points(n, 2)
    g, h = oracle.gh()
    dev = torch.device("cuda:0")
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a, np.uint64).view(np.int64)).to(dev)
    out = bp.batch_generate_range_proof(n, T(v), T(gam), T(sL), T(sR), T(rnd), T(G), T(H), T(g), T(h))
    batch = bp.RangeProofBatch(n, **{k: out[k] for k in bp.RangeProofBatch.FIELDS + ("taux", "mu")})
    ok = torch.zeros(B, dtype=torch.uint8, device=dev)
    bp.batch_range_proof_verify(batch, T(G), T(H), T(g), T(h), ok)
    torch.cuda.synchronize()
    o = {k: t.cpu().numpy().view(np.uint64) for k, t in out.items() if k not in ("valid", "_keep")}
    for p in range(B):
        head = np.concatenate([o[k][p] for k in ("V", "A", "S", "T1", "T2", "taux", "mu", "t", "c", "x")])
        okr, _, _, _, _ = oracle.cuda_range_proof_verify(head, o["V"][p], n, o["a"][p], o["b"][p], o["L"][p],
                                                         o["R"][p], G, H, g, h)
        assert bool(ok[p].item()) == okr, p


# ----------------------------------------------------------------------------- field arithmetic corners
M64 = (1 << 64) - 1
P_LIMBS = [0xFFFFFFFFFFFFFFED, M64, M64, 0x7FFFFFFFFFFFFFFF]
WRAP19 = 0x79435E50D79435E5                      # 19 * WRAP19 = 2^64 - 1 (mod 2^64)


def _lossy_sub_p(h):
    """curve25519_ops.cu:62-66 / :137-141: d_i = h_i - p_i - br; br = h_i < lo64(p_i + br)."""
    out, br = [], 0
    for i in range(4):
        out.append((h[i] - P_LIMBS[i] - br) & M64)
        br = int(h[i] < ((P_LIMBS[i] + br) & M64))
    return out


def _ge_p(h):
    for i in (3, 2, 1, 0):
        if h[i] != P_LIMBS[i]:
            return h[i] > P_LIMBS[i]
    return True


def _ref_fold(t):
    """curve25519_ops.cu:114-145 restated on Python ints (the reference's exact carry rules)."""
    h, cy = list(t[:4]), 0
    for i in range(4):
        c = (t[i + 4] * 19 + cy) & M64
        h[i] = (h[i] + c) & M64
        cy = int(h[i] < c)
    return _lossy_sub_p(h) if (cy or _ge_p(h)) else h


def test_fold_corners_vs_reference_rule(bp):
    """The product fold (device asm form) on crafted 512-bit inputs: 19 t_{i+4} = 2^64-1 with and without a
    carry in (the reference drops that carry), sums at and around p, carries out of the top limb."""
    import torch
    rng = np.random.default_rng(19)
    cands = [0, 1, 2, 18, 19, 20, M64, M64 - 1, WRAP19, WRAP19 - 1, WRAP19 + 1, P_LIMBS[0], P_LIMBS[0] - 1,
             P_LIMBS[3], 1 << 63, (1 << 63) - 1, 0xFFFFFFFF, 1 << 32]
    ts = []
    for k in range(4000):
        if k % 4 == 0:
            t = [int(x) for x in rng.integers(0, 2**63, 8, dtype=np.uint64) * 2 + rng.integers(0, 2, 8, dtype=np.uint64)]
        else:
            t = [cands[int(rng.integers(0, len(cands)))] if rng.random() < 0.7 else
                 int(rng.integers(0, 2**63, dtype=np.uint64)) * 2 for _ in range(8)]
        ts.append(t)
    ts.append([M64, M64, M64, M64, WRAP19, WRAP19, WRAP19, WRAP19])
    ts.append([M64 - 18, M64, M64, P_LIMBS[3], 0, 0, 0, 0])
    arr = np.array(ts, dtype=np.uint64)
    dev = torch.device("cuda:0")
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a).view(np.int64)).to(dev)
    r = torch.empty(len(ts), 4, dtype=torch.int64, device=dev)
    bp.field_op("fold", r, T(arr[:, :4]), T(arr[:, 4:]))
    torch.cuda.synchronize()
    got = r.cpu().numpy().view(np.uint64)
    for i, t in enumerate(ts):
        assert [int(x) for x in got[i]] == _ref_fold(t), (i, [hex(x) for x in t])


@pytest.mark.parametrize("op", ["mul", "sq"])
def test_bounded_product_gate(bp, oracle, op):
    """mul512 / sqr512 run the bounded products (tools/gen_mul_asm.py: the first carry of every
    column uncounted) unless a lane's gating words exceed 0xFFFFFFEF — mul: a[0] or b[7]; sq: a[0]
    or a[7] — when the wave runs the counting product.
    Waves here: (1) every gating word at or just under its bound with all other words 2^32 - 1 (the
    largest products the bounded forms meet); (2) one lane just over a bound at a rotating position
    among such lanes; (3) all-ones operands.  Every lane equals the oracle's fe25519_mul
    (== fe25519_sq, curve25519_ops.cu:93-149)."""
    import torch
    rng = np.random.default_rng(17 if op == "mul" else 18)
    LOW = 0xFFFFFFEF
    TOP = 0xFFFFFFEF

    def fe_words(words):
        return np.array([words[2 * k] | (words[2 * k + 1] << 32) for k in range(4)], np.uint64)
    a_l, b_l = [], []
    for w in range(64):
        for lane in range(64):
            aw = [0xFFFFFFFF if rng.random() < 0.7 else int(rng.integers(0, 2**32)) for _ in range(8)]
            bw = [0xFFFFFFFF if rng.random() < 0.7 else int(rng.integers(0, 2**32)) for _ in range(8)]
            aw[0] = LOW - int(rng.integers(0, 3))
            aw[7], bw[7] = TOP - int(rng.integers(0, 3)), TOP - int(rng.integers(0, 3))
            if 16 <= w < 56 and lane == (w * 37) % 64:   # one lane over a bound: the counting form
                which = w % 3
                if which == 0:
                    aw[0] = [LOW + 1, 0xFFFFFFFF][w % 2]
                elif which == 1:
                    aw[7] = [TOP + 1, 0xFFFFFFFF][w % 2]
                else:
                    bw[7] = [TOP + 1, 0xFFFFFFFF][w % 2]
            if w >= 56:
                aw = [0xFFFFFFFF] * 8
                bw = [0xFFFFFFFF] * 8
            a_l.append(fe_words(aw))
            b_l.append(fe_words(bw))
    a, b = np.stack(a_l), np.stack(b_l)
    if op == "sq":
        b = a.copy()
    dev = torch.device("cuda:0")
    T = lambda x: torch.from_numpy(np.ascontiguousarray(x).view(np.int64)).to(dev)
    r = torch.empty(len(a), 4, dtype=torch.int64, device=dev)
    if op == "sq":
        bp.field_op("sq", r, T(a))
    else:
        bp.field_op("mul", r, T(a), T(b))
    torch.cuda.synchronize()
    got = r.cpu().numpy().view(np.uint64)
    for i in range(len(a)):
        assert np.array_equal(got[i], oracle.fe_mul(a[i], b[i])), i


def test_quad_product_gate(bp, oracle):
    """fe_mul_q4 (ge25519_quad.h, the k_terms<4> / <16> drain forms' product split over a lane quad)
    runs the bounded 2x8 row products (mul2x8_bounded_asm) unless some lane's row word a[0] — x word
    0, 2, 4 or 6 — exceeds 0xFFFFFFEF, when the wave runs the counting mul2x8_asm.  Through
    field_op "mul_q4" (one element per quad, 16 per wave): (1) every row word at or just under the
    bound with all other words 2^32 - 1; (2) one element per wave with one row word just over the
    bound or 2^32 - 1, at a rotating row position; (3) all-ones operands.  Every element equals the
    oracle's fe25519_mul (curve25519_ops.cu:93-149)."""
    import torch
    rng = np.random.default_rng(19)
    LOW = 0xFFFFFFEF

    def fe_words(words):
        return np.array([words[2 * k] | (words[2 * k + 1] << 32) for k in range(4)], np.uint64)
    a_l, b_l = [], []
    for w in range(64):
        for el in range(16):
            aw = [0xFFFFFFFF if rng.random() < 0.7 else int(rng.integers(0, 2**32)) for _ in range(8)]
            bw = [0xFFFFFFFF if rng.random() < 0.7 else int(rng.integers(0, 2**32)) for _ in range(8)]
            for k in (0, 2, 4, 6):
                aw[k] = LOW - int(rng.integers(0, 3))
            if 8 <= w < 56 and el == (w * 7) % 16:   # one quad lane over the bound: the counting form
                aw[2 * (w % 4)] = [LOW + 1, 0xFFFFFFFF][(w // 4) % 2]
            if w >= 56:
                aw, bw = [0xFFFFFFFF] * 8, [0xFFFFFFFF] * 8
            a_l.append(fe_words(aw))
            b_l.append(fe_words(bw))
    a, b = np.stack(a_l), np.stack(b_l)
    dev = torch.device("cuda:0")
    T = lambda x: torch.from_numpy(np.ascontiguousarray(x).view(np.int64)).to(dev)
    r = torch.empty(len(a), 4, dtype=torch.int64, device=dev)
    bp.field_op("mul_q4", r, T(a), T(b))
    torch.cuda.synchronize()
    got = r.cpu().numpy().view(np.uint64)
    for i in range(len(a)):
        assert np.array_equal(got[i], oracle.fe_mul(a[i], b[i])), i


@pytest.mark.parametrize("op", ["mul_k", "mul_q4_k"])
def test_mul_by_k_vs_oracle(bp, oracle, op):
    """fe_mul_k (ge25519_dev.h: every point operation's C = (T1 T2) k, the product counting only the
    carries its column bounds allow, tools/gen_mul_asm.py k_columns) and its lane-quad split
    fe_mul_q4_k (the drain forms' C) equal the oracle's fe25519_mul(x, k) (curve25519_ops.cu:93-149,
    k = curve25519_ops.cu:341-346) for all-ones words (the partial sums' maximum), words at p and
    random values, through field_op "mul_k" / "mul_q4_k"."""
    import torch
    rng = np.random.default_rng(23)
    N = 4096
    x = rng.integers(0, 2**64, size=(N, 4), dtype=np.uint64)
    x[:64] = np.uint64(2**64 - 1)
    x[64:128] = np.array(P_LIMBS, np.uint64)
    x[128:192, 0] = np.uint64(2**64 - 1)
    x[192:256, 3] = np.uint64(2**64 - 1)
    k = np.array([0x75EB4DCA135978A3, 0x00700A4D4141D8AB, 0x8CC740797779E898, 0x52036CEE2B6FFE73], np.uint64)
    dev = torch.device("cuda:0")
    r = torch.empty(N, 4, dtype=torch.int64, device=dev)
    bp.field_op(op, r, torch.from_numpy(x.view(np.int64)).to(dev))
    torch.cuda.synchronize()
    got = r.cpu().numpy().view(np.uint64)
    for i in range(N):
        assert np.array_equal(got[i], oracle.fe_mul(x[i], k)), i


@pytest.mark.parametrize("kind", range(6))
def test_sha256_message_shapes_vs_fips(bp, oracle, kind):
    """The device SHA-256 of every message shape on the challenge path (sha256_dev.h: fixed layouts,
    register-resident) against hashlib (FIPS 180-4) over the same bytes: y / z / x challenges
    (bulletproof_challenge.cu:24-77), an inner-product round challenge (crv:185-205), the prover's
    13-byte-tag IPA transcript start (rp.cu:1636-1650, every field element at an unaligned offset)
    and the unmasked four-value digest (crv:330-344).  Field elements are random 256-bit words, so
    most are non-canonical: the hashed bytes are the host fe25519_tobytes (oracle) where the
    reference canonicalises, the raw limbs where it does not."""
    import hashlib
    import torch
    rng = np.random.default_rng(40 + kind)
    N = 300
    f = rng.integers(0, 2**64, size=(N, 6, 4), dtype=np.uint64)
    f[:8] = np.uint64(2**64 - 1)          # all-ones and at-p words among them
    f[8:16, :, :] = np.array(P_LIMBS, np.uint64)
    canon = lambda x: bytes(oracle.fe_tobytes(x))
    raw = lambda x: np.ascontiguousarray(x, np.uint64).tobytes()
    shapes = {
        0: lambda r: b"BulletproofYChal" + b"".join(canon(r[k]) for k in range(6)) + b"y_ch",
        1: lambda r: b"BulletproofZChal" + raw(r[0]) + b"z_ch",
        2: lambda r: b"BulletproofXChal" + b"".join(canon(r[k]) for k in range(4)) + b"xcha",
        3: lambda r: b"InnerProductChal" + raw(r[0]) + canon(r[1]) + canon(r[2]),
        4: lambda r: b"BulletproofIP" + canon(r[0]) + canon(r[1]) + canon(r[2]),
        5: lambda r: b"".join(raw(r[k]) for k in range(4)),
    }
    dev = torch.device("cuda:0")
    inp = torch.from_numpy(f.view(np.int64)).to(dev)
    out = torch.empty(N, 4, dtype=torch.int64, device=dev)
    bp.sha_probe(kind, out, inp)
    torch.cuda.synchronize()
    got = out.cpu().numpy().view(np.uint64)
    for i in range(N):
        d = bytearray(hashlib.sha256(shapes[kind](f[i])).digest())
        if kind != 5:
            d[31] &= 0x7F   # generate_challenge: output[31] &= 0x7F (bulletproof_challenge.cu:20)
        assert got[i].tobytes() == bytes(d), (kind, i)


def _edge_cases(op, rng):
    """Operand pairs that put one lane on each rare edge the field asm tests for (fe_add_asm /
    fe_sub_asm / fe_fold_asm in field_asm.h): every exact-form branch taken by exactly the case
    that needs it."""
    P0, P3 = P_LIMBS[0], P_LIMBS[3]
    r = lambda: int(rng.integers(0, 2**64, dtype=np.uint64))
    top = lambda: r() | (1 << 63)
    fix = [[r(), r(), M64, top()], [P0 + 3, r(), r(), top()], [P0, M64, M64, P3], [P0 + 18, M64, M64, P3],
           [P0 + 5, M64, r(), top()], [r(), r(), M64, P3], [M64, M64, M64, M64], [P0 - 1, r(), M64, top()]]
    out = []
    if op in ("add", "fold"):   # the fix-up's edges: b = 0 makes the sum / fold the edge vector itself
        out += [(f, [0, 0, 0, 0]) for f in fix]
    if op == "fold":            # x_i = 19 WRAP19 = 2^64 - 1: the reference's dropped carry
        for i in (1, 2, 3):
            for _ in range(3):
                hi = [r() if k != i else WRAP19 for k in range(4)]
                out.append(([r(), r(), r(), r()], hi))
    if op == "sub":
        for i in (1, 2, 3):     # g_i = 2^64 - 1: the lossy borrow
            for _ in range(3):
                out.append(([r(), r(), r(), r()], [r() if k != i else M64 for k in range(4)]))
        for t in ([5, r(), r(), 7], [18, r(), r(), 9], [0, r(), r(), 3], [r() | 0x100, M64, r(), 5],
                  [r() | 0x100, r(), M64, 6], [2, M64, M64, 1]):   # the "+ p" pass's edges, with a borrow
            g = [r(), r() & 0xFFFFFFFF7FFFFFFF, r() & 0xFFFFFFFF7FFFFFFF, 0xFFFFFFFFFFFFFFFE]
            tv = sum(x << (64 * k) for k, x in enumerate(t))
            gv = sum(x << (64 * k) for k, x in enumerate(g))
            av = (tv + gv) % (1 << 256)
            assert av < gv
            out.append(([(av >> (64 * k)) & M64 for k in range(4)], g))
    return out


@pytest.mark.parametrize("op", ["add", "sub", "fold", "mul", "addsub_add", "addsub_sub",
                                "add_lat", "add_defer", "fold_lat", "fold_defer", "addsub_lat_add", "addsub_lat_sub",
                                "addsub_defer_add", "addsub_defer_sub"])
def test_field_fast_forms_one_edge_lane_per_wave(bp, oracle, op):
    """The field asm runs a short form unless some lane of the wave sits on one of the rare edges
    (a limb or word equal to 2^64-1 / 2^32-1, t0 >= p0, t0 < 19): the exact form then runs for the
    whole wave.  Here each edge case sits alone in its own wave, at a rotating lane, among 63
    common lanes (the exact form must give those the same bits); further waves hold edge limbs at
    random, and the last ones near-edge values only (words 2^32-2, high words all ones with low
    words not) that the short form must get right.  The *_lat / *_defer ops run the 16-lane row
    step's latency forms and its deferred rare-edge test (a missed edge would leave a fast result
    the oracle rejects)."""
    import torch
    kind = op
    op = op.replace("_lat", "").replace("_defer", "")   # the operation the oracle checks
    rng = np.random.default_rng({"add": 1, "sub": 2, "fold": 3, "mul": 4, "addsub_add": 5, "addsub_sub": 6}[op] +
                                (10 if "_lat" in kind else 20 if "_defer" in kind else 0))
    # the fused add/sub block (fe_addsub_asm) takes its exact path when either op's edge fires, so
    # it gets both ops' edge cases whichever of its outputs is checked
    cases = _edge_cases(op, rng) if not op.startswith("addsub") else _edge_cases("add", rng) + _edge_cases("sub", rng)
    waves = len(cases) + 64
    N = 64 * waves
    a = rand_fe(rng, N, top=True)
    b = rand_fe(rng, N, top=True)
    for w, (f, g) in enumerate(cases):
        i = 64 * w + (w * 37) % 64
        a[i], b[i] = np.array(f, np.uint64), np.array(g, np.uint64)
    edges = [M64, M64 - 1, 0xFFFFFFFF00000000, 0x00000000FFFFFFFF, P_LIMBS[0], P_LIMBS[0] - 1, 18, 19, 0,
             P_LIMBS[3], 1 << 63, WRAP19, WRAP19 + 1, 0xFFFFFFFFFFFFFFEE]
    for w in range(len(cases), len(cases) + 32):   # one lane with edge limbs at random
        i = 64 * w + (w * 37) % 64
        for arr in (a, b):
            for limb in range(4):
                if rng.random() < 0.6:
                    arr[i, limb] = np.uint64(edges[int(rng.integers(0, len(edges)))])
    near = [0xFFFFFFFEFFFFFFFE, 0xFFFFFFFE00000000, 0xFFFFFFFF7FFFFFFF, 0x7FFFFFFFFFFFFFFE, 0xFFFFFFFEFFFFFFFF,
            20, 0x100000000, 0xFFFFFFFEFFFFFF00]
    for w in range(len(cases) + 32, waves):   # near-edge values only (the short form)
        for i in range(64 * w, 64 * w + 64):
            for arr in (a, b):
                for limb in range(4):
                    if rng.random() < 0.5:
                        arr[i, limb] = np.uint64(near[int(rng.integers(0, len(near)))])
    dev = torch.device("cuda:0")
    T = lambda x: torch.from_numpy(np.ascontiguousarray(x).view(np.int64)).to(dev)
    r = torch.empty(N, 4, dtype=torch.int64, device=dev)
    bp.field_op(kind, r, T(a), T(b))
    torch.cuda.synchronize()
    got = r.cpu().numpy().view(np.uint64)
    for i in range(N):
        if op == "fold":
            want = _ref_fold([int(x) for x in a[i]] + [int(x) for x in b[i]])
        else:
            want = [int(x) for x in getattr(oracle, "fe_" + op.replace("addsub_", ""))(a[i], b[i])]
        assert [int(x) for x in got[i]] == want, (kind, i, [hex(int(x)) for x in a[i]], [hex(int(x)) for x in b[i]])


def test_sq_matches_mul(bp, oracle):
    """Dedicated squaring (36 products) == fe25519_mul(x, x) on edge-heavy limbs."""
    import torch
    rng = np.random.default_rng(7)
    x = rng.integers(0, 2**64, size=(3000, 4), dtype=np.uint64)
    x[::3] = np.array([M64, M64, M64, M64], np.uint64)
    x[1::7, 1:3] = np.uint64(M64)
    dev = torch.device("cuda:0")
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a).view(np.int64)).to(dev)
    r = torch.empty(len(x), 4, dtype=torch.int64, device=dev)
    bp.field_op("sq", r, T(x))
    torch.cuda.synchronize()
    got = r.cpu().numpy().view(np.uint64)
    for i in range(0, len(x), 13):
        assert np.array_equal(got[i], oracle.fe_mul(x[i], x[i])), i


# ----------------------------------------------------------------------------- Pippenger (labelled alternative)
@pytest.mark.parametrize("n,c", [(1, 12), (2, 4), (17, 12), (300, 12), (1000, 8), (777, 4), (20000, 8), (4096, 12),
                                 (70000, 8),    # n > 65536: several histogram tiles per window
                                 (999, 5), (2048, 7), (3001, 11)])   # odd widths: partial top windows
def test_msm_pippenger_vs_oracle(bp, oracle, n, c):
    """hipbp_msm_pippenger == orc_msm_pippenger (the bucket algorithm restated in C): zero and short
    scalars (empty / crowded buckets), odd bucket sizes, every window width class."""
    import torch
    rng = np.random.default_rng(n * 31 + c)
    P = oracle.base_points(n, 9)
    s = rand_fe(rng, n)
    s[::7] = 0
    s[1::5, 1:] = 0
    if n > 100:
        s[3::11] = s[3]                          # a crowded bucket in every window
    dev = torch.device("cuda:0")
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a, np.uint64).view(np.int64)).to(dev)
    out = torch.zeros(16, dtype=torch.int64, device=dev)
    bp.msm_pippenger(out, T(s), T(P), c)
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy().view(np.uint64), oracle.msm_pippenger(s, P, c))


def test_msm_pippenger_concurrent_streams(bp, oracle):
    """Independent Pippenger MSMs in flight on two streams at once (per-stream workspaces, no
    host waits inside the call): every result equals the oracle's, whatever the interleaving."""
    import torch
    dev = torch.device("cuda:0")
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a, np.uint64).view(np.int64)).to(dev)
    cases = []
    for k, (n, c) in enumerate([(5000, 12), (3000, 8), (4096, 12), (1, 4)]):
        rng = np.random.default_rng(100 + k)
        P = oracle.base_points(n, 20 + k)
        s = rand_fe(rng, n)
        s[::9] = s[0]
        cases.append((T(s), T(P), c, oracle.msm_pippenger(s, P, c)))
    sts = [torch.cuda.Stream(dev) for _ in range(2)]
    outs = torch.zeros(3 * len(cases), 16, dtype=torch.int64, device=dev)
    for r in range(3):
        for k, (sd, Pd, c, _) in enumerate(cases):
            bp.msm_pippenger(outs[r * len(cases) + k], sd, Pd, c, stream=sts[(r + k) % 2])
    torch.cuda.synchronize()
    got = outs.cpu().numpy().view(np.uint64)
    for r in range(3):
        for k, (_, _, _, want) in enumerate(cases):
            assert np.array_equal(got[r * len(cases) + k], want), (r, k)


@pytest.mark.parametrize("n,count,c", [(300, 3, 12), (1000, 5, 8), (1, 4, 4), (4096, 2, 12), (777, 1, 4),
                                       (70001, 2, 12), (1002, 3, 12)])   # odd n: one key per thread
def test_msm_pippenger_batch_vs_oracle(bp, oracle, n, count, c):
    """hipbp_msm_pippenger_batch: count MSMs over the same points in one call, each equal to
    orc_msm_pippenger of its own scalars (shared sort / bucket trees / Horner launch)."""
    import torch
    rng = np.random.default_rng(n * 7 + count)
    P = oracle.base_points(n, 31)
    s = rand_fe(rng, count * n)
    s[::11] = 0
    if n > 100:
        s[5::13] = s[5]                           # crowded buckets across the MSMs
    dev = torch.device("cuda:0")
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a, np.uint64).view(np.int64)).to(dev)
    out = torch.zeros(count, 16, dtype=torch.int64, device=dev)
    bp.msm_pippenger_batch(out, T(s), T(P), c)
    torch.cuda.synchronize()
    got = out.cpu().numpy().view(np.uint64)
    for m in range(count):
        assert np.array_equal(got[m], oracle.msm_pippenger(s[m * n:(m + 1) * n], P, c)), m


def test_msm_pippenger_key_paths_agree(bp, oracle, monkeypatch):
    """The 32-bit-key sort (digit << ib | i, c + ib <= 32) and the 16-bit-key sort with
    counting-iterator values (forced by HIPBP_PIP_KEYS16=1; the path for larger n) give the same
    bits: single and batched calls, n % 4 == 0 and not, a crowded bucket per window."""
    import torch
    dev = torch.device("cuda:0")
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a, np.uint64).view(np.int64)).to(dev)
    for n, count, c in [(5000, 1, 12), (4097, 3, 8), (70000, 2, 12)]:
        rng = np.random.default_rng(n + c)
        P = oracle.base_points(n, 40)
        s = rand_fe(rng, count * n)
        s[::9] = s[0]
        outs = []
        for force in ("0", "1"):
            monkeypatch.setenv("HIPBP_PIP_KEYS16", force)
            out = torch.zeros(count, 16, dtype=torch.int64, device=dev)
            bp.msm_pippenger_batch(out, T(s), T(P), c)
            torch.cuda.synchronize()
            outs.append(out.cpu().numpy().view(np.uint64))
        assert np.array_equal(outs[0], outs[1]), (n, count, c)
        assert np.array_equal(outs[0][0], oracle.msm_pippenger(s[:n], P, c)), (n, count, c)


def test_msm_pippenger_tail_layers_agree(bp, oracle, monkeypatch):
    """The LDS tail from another layer (HIPBP_PIP_TAIL_LAYER: 1 = nearly every bucket summed in LDS,
    the whole-bucket staging measured in profiles/ab/r06ac; 6 = fewer buckets there) gives the
    oracle's bits: its 512-node chunks stay aligned to the canonical bucket tree."""
    import torch
    dev = torch.device("cuda:0")
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a, np.uint64).view(np.int64)).to(dev)
    for n, c in [(70000, 8), (20000, 12), (3001, 11)]:
        rng = np.random.default_rng(n + 3 * c)
        P = oracle.base_points(n, 41)
        s = rand_fe(rng, n)
        s[5::13] = s[5]   # a crowded bucket per window (a list longer than one chunk at n = 70000)
        want = oracle.msm_pippenger(s, P, c)
        for tl in ("1", "2", "6"):
            monkeypatch.setenv("HIPBP_PIP_TAIL_LAYER", tl)
            out = torch.zeros(16, dtype=torch.int64, device=dev)
            bp.msm_pippenger(out, T(s), T(P), c)
            torch.cuda.synchronize()
            assert np.array_equal(out.cpu().numpy().view(np.uint64), want), (n, c, tl)


def test_msm_pippenger_rejects_bad_window(bp):
    import torch
    dev = torch.device("cuda:0")
    z = torch.zeros(4, 16, dtype=torch.int64, device=dev)
    with pytest.raises(bp.BulletproofError):
        bp.msm_pippenger(torch.zeros(16, dtype=torch.int64, device=dev), torch.zeros(4, 4, dtype=torch.int64,
                                                                                      device=dev), z, 13)


@pytest.mark.parametrize("kind,n", [("same", 3000), ("zero", 3000), ("one_bit", 3000), ("same", 10000),
                                    ("one_bit", 9001),
                                    ("same", 140000)])   # LDS tail: a 547-node layer-4 list, two chunks
def test_msm_pippenger_degenerate_scalars(bp, oracle, kind, n):
    """Every point in one bucket per window (deep bucket trees, many empty buckets).  n > 4096: the
    lists are longer than one k_pip_bidfill piece (BID_PIECE), so the extra-piece queue runs."""
    import torch
    c = 8
    P = oracle.base_points(n, 12)
    s = np.zeros((n, 4), np.uint64)
    if kind == "same":
        s[:] = rand_fe(np.random.default_rng(5), 1)[0]
    elif kind == "one_bit":
        s[:, 2] = np.uint64(1) << np.uint64(17)
    dev = torch.device("cuda:0")
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a, np.uint64).view(np.int64)).to(dev)
    out = torch.zeros(16, dtype=torch.int64, device=dev)
    bp.msm_pippenger(out, T(s), T(P), c)
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy().view(np.uint64), oracle.msm_pippenger(s, P, c))


@pytest.mark.parametrize("n,c", [(512, 12), (450, 12), (550, 12), (30, 8), (7, 5)])
def test_msm_pippenger_sparse_buckets_all_apis(bp, oracle, n, c):
    """n ~ 0.1-0.13 * 2^c: most buckets hold 0 or 1 point, so the padded step-0 layout has fewer
    than nb / 4 groups of lanes but up to nb / 8 groups — the octet tail path's lane count at step
    0.  Single call, a batch of 3 and a window split against the oracle."""
    import torch
    dev = torch.device("cuda:0")
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a, np.uint64).view(np.int64)).to(dev)
    rng = np.random.default_rng(n * 13 + c)
    P = oracle.base_points(n, 17)
    count = 3
    s = rand_fe(rng, count * n)
    want = [oracle.msm_pippenger(s[m * n:(m + 1) * n], P, c) for m in range(count)]
    out = torch.zeros(16, dtype=torch.int64, device=dev)
    bp.msm_pippenger(out, T(s[:n]), T(P), c)
    bo = torch.zeros(count, 16, dtype=torch.int64, device=dev)
    bp.msm_pippenger_batch(bo, T(s), T(P), c)
    W = (256 + c - 1) // c
    Sw = torch.zeros(W, 16, dtype=torch.int64, device=dev)
    h = W // 2
    bp.msm_pippenger_windows(Sw, T(s[:n]), T(P), 0, h, c)
    bp.msm_pippenger_windows(Sw, T(s[:n]), T(P), h, W, c)
    wo = torch.zeros(1, 16, dtype=torch.int64, device=dev)
    bp.msm_pippenger_horner(wo, Sw, c)
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy().view(np.uint64), want[0])
    got = bo.cpu().numpy().view(np.uint64)
    for m in range(count):
        assert np.array_equal(got[m], want[m]), m
    assert np.array_equal(wo.cpu().numpy().view(np.uint64)[0], want[0])
    assert np.array_equal(Sw.cpu().numpy().view(np.uint64), oracle.pippenger_windows(s[:n], P, c, 0, W))


# ----------------------------------------------------------------------------- batched MSM
@pytest.mark.parametrize("n,count", [(1, 3), (17, 5), (300, 4), (256, 2)])
def test_msm_batch_matches_single(bp, oracle, n, count):
    """hipbp_msm_batch: each of count MSMs over the same points == the oracle's canonical MSM."""
    import torch
    rng = np.random.default_rng(n + count)
    P = oracle.base_points(n, 13)
    s = rand_fe(rng, n * count)
    s[::9] = 0
    dev = torch.device("cuda:0")
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a, np.uint64).view(np.int64)).to(dev)
    out = torch.zeros(count, 16, dtype=torch.int64, device=dev)
    bp.msm_batch(out, T(s), T(P))
    torch.cuda.synchronize()
    out = out.cpu().numpy().view(np.uint64)
    for k in range(count):
        assert np.array_equal(out[k], oracle.msm_canon(s[k * n:(k + 1) * n], P)), k


def test_msm_batch_ipa4096_commitment(bp, golden, oracle):
    """configs[3]'s P = MSM(a||b, G||H) over 8192 points, for 3 proofs at once, equals the
    reference's P recorded in ipa4096.npz."""
    import os
    import sys
    import torch
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "golden"))
    from make_golden import ipa_vectors
    d, n, G, H, Q = _ipa4096(golden, oracle)
    a, b = ipa_vectors(n)
    sc = np.concatenate([a, b] * 3)
    dev = torch.device("cuda:0")
    T = lambda x: torch.from_numpy(np.ascontiguousarray(x, np.uint64).view(np.int64)).to(dev)
    out = torch.zeros(3, 16, dtype=torch.int64, device=dev)
    bp.msm_batch(out, T(sc), T(np.concatenate([G, H])))
    torch.cuda.synchronize()
    for k in range(3):
        assert np.array_equal(out.cpu().numpy().view(np.uint64)[k], d["P"])


def test_pipeline_sorted_and_unsorted_batches_in_flight(bp, oracle):
    """Lane-sorted (B >= 64) and index-order (B < 64) batches share ticks: every proof's verdict,
    P and check point equal the oracle's, whatever batch order and tick they ride in."""
    import torch
    from cudabulletproof_amd import synth
    n = 16
    G, H = oracle.base_points(n, 1), oracle.base_points(n, 2)
    g, h = oracle.gh()
    dev = torch.device("cuda:0")
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a, np.uint64).view(np.int64)).to(dev)
    pipe = bp.VerifyPipeline(130, n, T(G), T(H), T(h))
    outs = []
    for i, B in enumerate((100, 5, 130, 64, 3)):
        arrays = synth.proofs(B, n, seed=700 + i)
        batch = bp.RangeProofBatch.from_numpy(n, arrays, dev)
        ok = torch.zeros(B, dtype=torch.uint8, device=dev)
        P = torch.zeros(B, 16, dtype=torch.int64, device=dev)
        chk = torch.zeros(B, 16, dtype=torch.int64, device=dev)
        pipe.push(batch, ok, P, chk)
        outs.append((arrays, ok, P, chk, batch))
    pipe.flush()
    torch.cuda.synchronize()
    for arrays, ok, P, chk, _ in outs:
        B = len(arrays["t"])
        ok, P, chk = ok.cpu().numpy().astype(bool), P.cpu().numpy().view(np.uint64), chk.cpu().numpy().view(np.uint64)
        for p in range(0, B, 7):   # a sample of each batch
            head = np.concatenate([arrays[k][p] for k in ("V", "A", "S", "T1", "T2")] +
                                  [np.zeros(8, np.uint64), arrays["t"][p], arrays["c"][p], arrays["x"][p]])
            okr, Pr, chkr, _, _ = oracle.cuda_range_proof_verify(head, arrays["V"][p], n, arrays["a"][p],
                                                                 arrays["b"][p], arrays["L"][p], arrays["R"][p],
                                                                 G, H, g, h)
            assert ok[p] == okr and np.array_equal(P[p], Pr), (B, p)
            if okr:
                assert np.array_equal(chk[p], chkr), (B, p)
    pipe.close()


# ----------------------------------------------------------------------------- empty inputs
def test_empty_inputs_are_noops(bp):
    """n = 0 / count = 0 through every entry point: no launch, no fault, outputs untouched
    (the reference's n = 0 behaviour is an invalid 0-block launch; this is the defined form)."""
    import ctypes
    import torch
    dev = torch.device("cuda:0")
    out = np.full(16, 7, np.uint64)
    z4, z16 = np.zeros((0, 4), np.uint64), np.zeros((0, 16), np.uint64)
    sv, pv = bp.FieldVector(z4.ctypes.data, 0), bp.PointVector(z16.ctypes.data, 0)
    bp.lib().cuda_point_vector_multi_scalar_mul(ctypes.c_void_p(out.ctypes.data), ctypes.byref(sv), ctypes.byref(pv))
    assert (out == 7).all()
    r = torch.full((16,), 7, dtype=torch.int64, device=dev)
    e4 = torch.zeros(0, 4, dtype=torch.int64, device=dev)
    e16 = torch.zeros(0, 16, dtype=torch.int64, device=dev)
    bp.msm(r, e4, e16)
    bp.msm_pippenger(r, e4, e16, 12)
    bp.point_tree(r, e16)
    bp.msm_batch(torch.zeros(0, 16, dtype=torch.int64, device=dev), e4, torch.zeros(3, 16, dtype=torch.int64, device=dev))
    torch.cuda.synchronize()
    assert (r.cpu() == 7).all()
    from cudabulletproof_amd import synth
    arrays = {k: v[:0] for k, v in synth.proofs(1, 16, seed=1).items()}
    batch = bp.RangeProofBatch.from_numpy(16, arrays, dev)
    G, H = torch.zeros(16, 16, dtype=torch.int64, device=dev), torch.zeros(16, 16, dtype=torch.int64, device=dev)
    g = torch.zeros(16, dtype=torch.int64, device=dev)
    bp.batch_range_proof_verify(batch, G, H, g, g, torch.zeros(0, dtype=torch.uint8, device=dev))
    torch.cuda.synchronize()


# ----------------------------------------------------------------------------- concurrency / lifetimes
def test_msm_on_two_streams_at_once(bp, oracle):
    """hipbp_msm / hipbp_msm_batch / hipbp_point_tree on two torch streams with no sync between
    them, plus a Part-1 MSM on the engine stream in the middle: each stream has its own
    workspace, so every result equals the serial (oracle) one."""
    import torch
    dev = torch.device("cuda:0")
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a, np.uint64).view(np.int64)).to(dev)
    rng = np.random.default_rng(77)
    n1, n2, n3 = 3000, 1100, 300
    P1, P2, P3 = oracle.base_points(n1, 21), oracle.base_points(n2, 22), oracle.base_points(n3, 23)
    s1, s2, s3 = rand_fe(rng, n1), rand_fe(rng, 3 * n2), rand_fe(rng, n3)
    d1, d2, dp1, dp2 = T(s1), T(s2), T(P1), T(P2)
    torch.cuda.synchronize()
    st_a, st_b = torch.cuda.Stream(), torch.cuda.Stream()
    r1 = torch.zeros(16, dtype=torch.int64, device=dev)
    r2 = torch.zeros(3, 16, dtype=torch.int64, device=dev)
    rt = torch.zeros(16, dtype=torch.int64, device=dev)
    for _ in range(2):
        bp.msm(r1, d1, dp1, stream=st_a)
        bp.msm_batch(r2, d2, dp2, stream=st_b)
        r3 = bp.cuda_point_vector_multi_scalar_mul(s3, P3)   # engine stream, synchronous
        bp.point_tree(rt, dp1, stream=st_b)
    torch.cuda.synchronize()
    assert np.array_equal(r1.cpu().numpy().view(np.uint64), oracle.msm_canon(s1, P1))
    out2 = r2.cpu().numpy().view(np.uint64)
    for k in range(3):
        assert np.array_equal(out2[k], oracle.msm_canon(s2[k * n2:(k + 1) * n2], P2)), k
    assert np.array_equal(r3, oracle.msm_canon(s3, P3))
    rt_ref = torch.zeros(16, dtype=torch.int64, device=dev)
    bp.point_tree(rt_ref, dp1)
    torch.cuda.synchronize()
    assert np.array_equal(rt.cpu().numpy(), rt_ref.cpu().numpy())


def test_pipeline_mode2_batch_overwritten_after_push(bp, oracle):
    """range_proof_verify pipeline (mode 2): stage 0 runs a tick after the push, yet a batch is
    consumed by its own push — the caller refills the batch tensors right after each push and
    every result still equals the oracle's on the original proofs."""
    import torch
    from cudabulletproof_amd import synth
    n, B = 16, 12
    G, H = oracle.base_points(n, 1), oracle.base_points(n, 2)
    g, h = oracle.gh()
    dev = torch.device("cuda:0")
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a, np.uint64).view(np.int64)).to(dev)
    pipe = bp.VerifyPipeline(B, n, T(G), T(H), T(h), range_mode=2, g=T(g))
    rng = np.random.default_rng(5)
    runs = []
    for i in range(3):
        arrays = synth.proofs(B, n, seed=900 + i)
        arrays["taux"] = rand_fe(rng, B, top=False)
        arrays["mu"] = rand_fe(rng, B, top=False)
        batch = bp.RangeProofBatch.from_numpy(n, arrays, dev)
        outs = (torch.zeros(B, dtype=torch.uint8, device=dev), torch.zeros(B, 16, dtype=torch.int64, device=dev),
                torch.zeros(B, 16, dtype=torch.int64, device=dev), torch.zeros(B, dtype=torch.uint8, device=dev),
                torch.zeros(B, 4, 16, dtype=torch.int64, device=dev))
        pipe.push(batch, outs[0], outs[1], outs[2], flags_out=outs[3], poly_out=outs[4])
        for k in bp.RangeProofBatch.FIELDS + ("taux", "mu"):   # same stream, after the push
            getattr(batch, k).fill_(0x5A5A)
        runs.append((arrays, outs))
    pipe.flush()
    torch.cuda.synchronize()
    u = lambda t: t.cpu().numpy().view(np.uint64)
    for arrays, (ok, P, chk, fl, poly) in runs:
        heads = np.concatenate([arrays[k] for k in ("V", "A", "S", "T1", "T2", "taux", "mu", "t", "c", "x")], axis=1)
        res = (ok.cpu().numpy().astype(bool), u(P), u(chk), fl.cpu().numpy(), u(poly))
        _check_std_vs_oracle(oracle, n, arrays, heads, G, H, g, h, res)
    pipe.close()


@pytest.mark.parametrize("n,B,mode,K", [(16, 70, 1, 8), (64, 66, 1, 12), (16, 9, 2, 5), (64, 64, 2, 10),
                                        (4, 5, 1, 1), (16, 6, 0, 9)])
def test_pipeline_prefix_tables_same_bits(bp, oracle, n, B, mode, K):
    """hipbp_pipeline_prefix_tables: the generators' scalar multiplications start from a table
    entry at bit 255 - K; every output (verdict, P, check point, mode-2 flags and polynomial
    sides) is bit-identical to the table-free pipeline, and a sample equals the oracle."""
    import torch
    from cudabulletproof_amd import synth
    G, H = oracle.base_points(n, 1), oracle.base_points(n, 2)
    g, h = oracle.gh()
    dev = torch.device("cuda:0")
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a, np.uint64).view(np.int64)).to(dev)
    arrays = synth.proofs(B, n, seed=40 + n + K)
    rng = np.random.default_rng(K)
    arrays["taux"] = rand_fe(rng, B, top=False)
    arrays["mu"] = rand_fe(rng, B, top=False)
    arrays["t"][0] = 0                              # zero scalar: the dtab path beside the table path
    arrays["t"][1, 3] = np.uint64(1) << np.uint64(63 - K)   # exactly K leading zeros
    arrays["t"][1, :3] = 0
    arrays["a"][:, 0] = arrays["t"]
    arrays["c"][:] = arrays["t"]
    Pg = T(oracle.base_points(B, 9))                # mode 0: given P
    outs = []
    for bits in (0, K):
        pipe = bp.VerifyPipeline(B, n, T(G), T(H), T(h), range_mode=mode, g=T(g) if mode == 2 else None)
        if bits:
            pipe.prefix_tables(bits)
        batch = bp.RangeProofBatch.from_numpy(n, arrays, dev)
        o = [torch.zeros(B, dtype=torch.uint8, device=dev), torch.zeros(B, 16, dtype=torch.int64, device=dev),
             torch.zeros(B, 16, dtype=torch.int64, device=dev), torch.zeros(B, dtype=torch.uint8, device=dev),
             torch.zeros(B, 4, 16, dtype=torch.int64, device=dev)]
        if mode == 0:
            pipe.push(batch, o[0], None, o[2], P_in=Pg)
        elif mode == 1:
            pipe.push(batch, o[0], o[1], o[2])
        else:
            pipe.push(batch, o[0], o[1], o[2], flags_out=o[3], poly_out=o[4])
        pipe.flush()
        torch.cuda.synchronize()
        outs.append([x.cpu() for x in o])
        pipe.close()
    for a, b in zip(*outs):
        assert torch.equal(a, b)
    if mode == 1:
        ok, P = outs[1][0].numpy().astype(bool), outs[1][1].numpy().view(np.uint64)
        for p in range(0, B, 5):
            head = np.concatenate([arrays[k][p] for k in ("V", "A", "S", "T1", "T2")] +
                                  [np.zeros(8, np.uint64), arrays["t"][p], arrays["c"][p], arrays["x"][p]])
            okr, Pr, _, _, _ = oracle.cuda_range_proof_verify(head, arrays["V"][p], n, arrays["a"][p], arrays["b"][p],
                                                              arrays["L"][p], arrays["R"][p], G, H, g, h)
            assert ok[p] == okr and np.array_equal(P[p], Pr), p


def _pipeline_outputs(bp, n, B, mode, arrays, G, H, g, h, Pg, bits=0, gens=None, pushes=1):
    """One pipeline over `pushes` copies of the batch: ok, P, check, flags, poly of the last."""
    import torch
    dev = torch.device("cuda:0")
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a, np.uint64).view(np.int64)).to(dev)
    pipe = bp.VerifyPipeline(B, n, T(G), T(H), T(h), range_mode=mode, g=T(g) if mode == 2 else None)
    if gens is not None:
        pipe.use_gens(gens)
    elif bits:
        pipe.prefix_tables(bits)
    batch = bp.RangeProofBatch.from_numpy(n, arrays, dev)
    res = []
    for _ in range(pushes):
        o = [torch.zeros(B, dtype=torch.uint8, device=dev), torch.zeros(B, 16, dtype=torch.int64, device=dev),
             torch.zeros(B, 16, dtype=torch.int64, device=dev), torch.zeros(B, dtype=torch.uint8, device=dev),
             torch.zeros(B, 4, 16, dtype=torch.int64, device=dev)]
        if mode == 0:
            pipe.push(batch, o[0], None, o[2], P_in=Pg)
        elif mode == 1:
            pipe.push(batch, o[0], o[1], o[2])
        else:
            pipe.push(batch, o[0], o[1], o[2], flags_out=o[3], poly_out=o[4])
        res.append(o)
    pipe.flush()
    torch.cuda.synchronize()
    pipe.close()
    return [[x.cpu() for x in o] for o in res]


def _sample_vs_oracle(oracle, n, B, arrays, ok, P, G, H, g, h, step=5):
    for p in range(0, B, step):
        head = np.concatenate([arrays[k][p] for k in ("V", "A", "S", "T1", "T2")] +
                              [np.zeros(8, np.uint64), arrays["t"][p], arrays["c"][p], arrays["x"][p]])
        okr, Pr, _, _, _ = oracle.cuda_range_proof_verify(head, arrays["V"][p], n, arrays["a"][p], arrays["b"][p],
                                                          arrays["L"][p], arrays["R"][p], G, H, g, h)
        assert ok[p] == okr and np.array_equal(P[p], Pr), p


@pytest.mark.parametrize("n,B,mode,K,pushes", [(16, 70, 1, 0, 1), (64, 66, 1, 12, 2), (16, 9, 2, 5, 1),
                                               (64, 20, 2, 0, 3), (4, 5, 1, 1, 1), (16, 6, 0, 9, 2),
                                               (1, 3, 1, 0, 1), (64, 1, 1, 0, 1)])
def test_pipeline_quad_ticks_same_bits(bp, oracle, monkeypatch, n, B, mode, K, pushes):
    """The drain-tick forms — k_terms<4> (every scalar multiplication on a lane quad, sm_quad, the
    chains too), k_terms<2> (lane pairs, sm_pair) and k_terms<16> (16-lane rows, sm_row, the chains
    on quads) — forced on every tick (HIPBP_QUAD=1 / 2 / 3) give
    bit-identical verdicts, P, check points, mode-2 flags and polynomial sides to the lane form
    forced everywhere (HIPBP_QUAD=0): every region kind, with and without prefix tables, batches in
    flight together; a sample equals the oracle."""
    from cudabulletproof_amd import synth
    G, H = oracle.base_points(n, 1), oracle.base_points(n, 2)
    g, h = oracle.gh()
    arrays = synth.proofs(B, n, seed=70 + n + K + B)
    rng = np.random.default_rng(B + K)
    arrays["taux"] = rand_fe(rng, B, top=False)
    arrays["mu"] = rand_fe(rng, B, top=False)
    arrays["t"][0] = 0                                  # zero scalar: 256 identity doublings
    if B > 2:
        arrays["x"][1, 1:] = 0                           # a short fold scalar: long leading-zero run
    arrays["a"][:, 0] = arrays["t"]
    arrays["c"][:] = arrays["t"]
    import torch
    Pg = torch.from_numpy(oracle.base_points(B, 9).view(np.int64)).to("cuda:0")
    outs = []
    for q in ("0", "1", "2", "3"):   # lanes, quads, pairs, 16-lane rows on every tick
        monkeypatch.setenv("HIPBP_QUAD", q)
        outs.append(_pipeline_outputs(bp, n, B, mode, arrays, G, H, g, h, Pg, bits=K, pushes=pushes))
    for other in outs[1:]:
        for oa, ob in zip(outs[0], other):
            for a, b in zip(oa, ob):
                assert torch.equal(a, b)
    if mode == 1:
        o = outs[1][-1]
        _sample_vs_oracle(oracle, n, B, arrays, o[0].numpy().astype(bool), o[1].numpy().view(np.uint64), G, H, g, h)


@pytest.mark.parametrize("n,B,mode,K,pushes,q", [(64, 70, 1, 12, 3, None), (16, 130, 1, 0, 2, None),
                                                  (64, 9, 2, 5, 2, None), (16, 6, 2, 0, 1, "1"),
                                                  (64, 40, 1, 0, 2, "2"), (4, 5, 1, 3, 1, None),
                                                  (1, 3, 1, 0, 1, None), (64, 1, 1, 9, 1, "1")])
def test_pipeline_deferred_msm_same_bits(bp, oracle, monkeypatch, n, B, mode, K, pushes, q):
    """Split stage 0 (hipbp_pipeline_defer_msm: the MSM terms, t*h and c*Q as RK_MSMT chunks inside
    the batch's own fold-round ticks, stages 2 .. L, on the pipeline's stream; the lane trees at
    msm_last(L) + 1, the final-terms tick) gives the unsplit pipeline's verdicts, P, check points,
    mode-2 flags and polynomial sides bit for bit: batches in flight together, with and without
    prefix tables, each tick form; a sample equals the oracle."""
    from cudabulletproof_amd import synth
    import torch
    G, H = oracle.base_points(n, 1), oracle.base_points(n, 2)
    g, h = oracle.gh()
    arrays = synth.proofs(B, n, seed=1300 + n + B)
    rng = np.random.default_rng(B + n)
    arrays["taux"] = rand_fe(rng, B, top=False)
    arrays["mu"] = rand_fe(rng, B, top=False)
    arrays["t"][0] = 0
    arrays["a"][:, 0] = arrays["t"]
    arrays["c"][:] = arrays["t"]
    if q is not None:
        monkeypatch.setenv("HIPBP_QUAD", q)
    monkeypatch.delenv("HIPBP_DEFER_MSM", raising=False)
    want = _pipeline_outputs(bp, n, B, mode, arrays, G, H, g, h, None, bits=K, pushes=pushes)
    monkeypatch.setenv("HIPBP_DEFER_MSM", "1")
    got = _pipeline_outputs(bp, n, B, mode, arrays, G, H, g, h, None, bits=K, pushes=pushes)
    for oa, ob in zip(want, got):
        for a, b in zip(oa, ob):
            assert torch.equal(a, b)
    if mode == 1:
        o = got[-1]
        _sample_vs_oracle(oracle, n, B, arrays, o[0].numpy().astype(bool), o[1].numpy().view(np.uint64), G, H, g, h,
                          step=7)


def test_pipeline_defer_msm_api(bp, oracle):
    """The C-ABI switch: refused where the split does not apply (inner-product mode; n above the
    lane-tree limit), accepted in range mode, and a batch pushed with it verifies as without."""
    import torch
    from cudabulletproof_amd import synth
    dev = torch.device("cuda:0")
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a, np.uint64).view(np.int64)).to(dev)
    for n, mode, ok in ((64, 1, True), (64, 0, False), (128, 1, False), (16, 2, True)):
        G, H = oracle.base_points(n, 1), oracle.base_points(n, 2)
        g, h = oracle.gh()
        pl = bp.VerifyPipeline(8, n, T(G), T(H), T(h), range_mode=mode, g=T(g))
        if ok:
            pl.defer_msm(True)
            pl.defer_msm(False)
            pl.defer_msm(True)
        else:
            with pytest.raises(bp.BulletproofError):
                pl.defer_msm(True)
        pl.close()
    n = 64
    G, H = oracle.base_points(n, 1), oracle.base_points(n, 2)
    g, h = oracle.gh()
    arrays = synth.proofs(8, n, seed=77)
    batch = bp.RangeProofBatch.from_numpy(n, arrays, dev)
    outs = []
    for d in (False, True):
        pl = bp.VerifyPipeline(8, n, T(G), T(H), T(h))
        pl.defer_msm(d)
        ok = torch.zeros(8, dtype=torch.uint8, device=dev)
        P = torch.zeros(8, 16, dtype=torch.int64, device=dev)
        pl.push(batch, ok, P)
        pl.flush()
        torch.cuda.synchronize()
        pl.close()
        outs.append((ok.cpu(), P.cpu()))
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])


def test_pipeline_defer_msm_largest_lane_tree_n(bp, oracle, monkeypatch):
    """With the lane-tree limit raised (HIPBP_LANE_TREE_MAX = 4096) the split applies up to n = 512,
    whose split ticks hold 2 log2 n + 5 = 23 regions (<= the kernel's 24), and verifies as without
    it, 16 batches in flight; at n = 1024 (25 regions) the switch is refused with a message
    instead of a push failing on the region list (advisor r04)."""
    import torch
    from cudabulletproof_amd import synth
    monkeypatch.setenv("HIPBP_LANE_TREE_MAX", "4096")
    dev = torch.device("cuda:0")
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a, np.uint64).view(np.int64)).to(dev)
    n = 1024
    G, H = oracle.base_points(n, 1), oracle.base_points(n, 2)
    g, h = oracle.gh()
    pl = bp.VerifyPipeline(2, n, T(G), T(H), T(h))
    with pytest.raises(bp.BulletproofError, match="n <= 512"):
        pl.defer_msm(True)
    pl.close()
    n, B = 512, 2
    G, H = oracle.base_points(n, 1), oracle.base_points(n, 2)
    outs = []
    for d in (False, True):
        pl = bp.VerifyPipeline(B, n, T(G), T(H), T(h))
        pl.defer_msm(d)
        res = []
        for k in range(16):   # more batches than stages: steady-state ticks with every stage's regions
            batch = bp.RangeProofBatch.from_numpy(n, synth.proofs(B, n, seed=900 + k), dev)
            ok = torch.zeros(B, dtype=torch.uint8, device=dev)
            P = torch.zeros(B, 16, dtype=torch.int64, device=dev)
            pl.push(batch, ok, P)
            res.append((ok, P, batch))
        pl.flush()
        torch.cuda.synchronize()
        pl.close()
        outs.append([(ok.cpu(), P.cpu()) for ok, P, _ in res])
    for (a, b), (c, e) in zip(outs[0], outs[1]):
        assert torch.equal(a, c) and torch.equal(b, e)


@pytest.mark.parametrize("n,B,lt", [(512, 3, "1024"), (512, 3, "512"), (256, 4, "4096"), (64, 5, "0")])
def test_pipeline_lane_tree_knob_same_bits(bp, oracle, monkeypatch, n, B, lt):
    """HIPBP_LANE_TREE_MAX only moves the MSM trees between RK_LTREE (one lane / quad per proof)
    and RK_TREE blocks: with the lane trees on for n > 256 (above the block size) P and the
    verdicts are the default layout's and the oracle's (advisor r03: final_task once re-reduced
    the finished lane-tree root with the chunk roots there)."""
    from cudabulletproof_amd import synth
    import torch
    G, H = oracle.base_points(n, 1), oracle.base_points(n, 2)
    g, h = oracle.gh()
    arrays = synth.proofs(B, n, seed=900 + n)
    monkeypatch.delenv("HIPBP_LANE_TREE_MAX", raising=False)
    want = _pipeline_outputs(bp, n, B, 1, arrays, G, H, g, h, None)
    monkeypatch.setenv("HIPBP_LANE_TREE_MAX", lt)
    got = _pipeline_outputs(bp, n, B, 1, arrays, G, H, g, h, None)
    for a, b in zip(want[-1], got[-1]):
        assert torch.equal(a, b)
    _sample_vs_oracle(oracle, n, B, arrays, got[-1][0].numpy().astype(bool), got[-1][1].numpy().view(np.uint64),
                      G, H, g, h, step=1)


@pytest.mark.parametrize("n,B,K", [(16, 70, 22), (16, 70, 23), (64, 40, 20), (64, 40, 21)])
def test_pipeline_headline_table_width_same_bits(bp, oracle, n, B, K):
    """The headline's table width (bench.py DEFAULT_PREFIX_BITS: K = 21 at n = 64, 34.9 GB; round 4
    ran K = 23): prefix tables of K = 20-23 bits through a generator set (as bench.py uses them) give
    the table-free pipeline's bits, and a sample equals the oracle (n = 16 at K = 22 / 23: 18 / 36 GB
    of tables; n = 64 at K = 20 / 21: 17 / 35 GB)."""
    import torch
    from cudabulletproof_amd import synth
    dev = torch.device("cuda:0")
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a, np.uint64).view(np.int64)).to(dev)
    G, H = oracle.base_points(n, 1), oracle.base_points(n, 2)
    g, h = oracle.gh()
    arrays = synth.proofs(B, n, seed=300 + K)
    arrays["t"][0] = 0
    arrays["t"][1, 3] = np.uint64(1) << np.uint64(63 - K)   # exactly K leading zeros
    arrays["t"][1, :3] = 0
    arrays["a"][:, 0] = arrays["t"]
    arrays["c"][:] = arrays["t"]
    plain = _pipeline_outputs(bp, n, B, 1, arrays, G, H, g, h, None, pushes=2)
    gens = bp.Generators(n, T(G), T(H), T(g), T(h), prefix_bits=K)
    tab = _pipeline_outputs(bp, n, B, 1, arrays, G, H, g, h, None, gens=gens, pushes=2)
    gens.close()
    torch.cuda.empty_cache()
    for oa, ob in zip(plain, tab):
        for a, b in zip(oa, ob):
            assert torch.equal(a, b)
    o = tab[-1]
    _sample_vs_oracle(oracle, n, B, arrays, o[0].numpy().astype(bool), o[1].numpy().view(np.uint64), G, H, g, h,
                      step=7)


@pytest.mark.parametrize("n,K", [(16, 0), (16, 12), (64, 16)])
def test_batch_verify_gens_matches_plain(bp, golden, n, K):
    """hipbp_batch_range_proof_verify_gens (a generator set's generators and K-bit prefix tables,
    one-shot) gives the plain one-shot call's verdicts, P and check points: the reference proofs
    (their verdicts, P, check points) and 300 synthetic ones; the plain call after it still runs
    without tables (the lent tables go back); a batch of another n is refused."""
    import torch
    from cudabulletproof_amd import synth
    from oracle import pyoracle
    d = golden(f"proofs_n{n}")
    dev = torch.device("cuda:0")
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a, np.uint64).view(np.int64)).to(dev)
    gens = bp.Generators(n, T(d["G"]), T(d["H"]), T(d["g"]), T(d["h"]), prefix_bits=K)
    try:
        hs = [pyoracle.head_fields(h) for h in d["head"]]
        ref = dict(V=d["V"], A=np.stack([h["A"] for h in hs]), S=np.stack([h["S"] for h in hs]),
                   T1=np.stack([h["T1"] for h in hs]), T2=np.stack([h["T2"] for h in hs]),
                   t=np.stack([h["t"] for h in hs]), a=d["a"], b=d["b"], c=np.stack([h["c"] for h in hs]),
                   x=np.stack([h["x"] for h in hs]), L=d["L"], R=d["R"])
        for arrays in (ref, synth.proofs(300, n, seed=70 + K)):
            batch = bp.RangeProofBatch.from_numpy(n, arrays, dev)
            outs = []
            for use in (False, True, False):
                ok = torch.zeros(batch.count, dtype=torch.uint8, device=dev)
                P = torch.zeros(batch.count, 16, dtype=torch.int64, device=dev)
                chk = torch.zeros(batch.count, 16, dtype=torch.int64, device=dev)
                if use:
                    bp.batch_range_proof_verify_gens(batch, gens, ok, P, chk)
                else:
                    bp.batch_range_proof_verify(batch, T(d["G"]), T(d["H"]), T(d["g"]), T(d["h"]), ok, P, chk)
                torch.cuda.synchronize()
                outs.append([x.cpu() for x in (ok, P, chk)])
            for o in outs[1:]:
                for a, b in zip(outs[0], o):
                    assert torch.equal(a, b)
            if arrays is ref:
                assert np.array_equal(outs[1][0].numpy().astype(bool), d["ok_cuda"].astype(bool))
                assert np.array_equal(outs[1][1].numpy().view(np.uint64), d["P"])
                assert np.array_equal(outs[1][2].numpy().view(np.uint64), d["check"])
        other = bp.RangeProofBatch.from_numpy(2 * n, synth.proofs(2, 2 * n, seed=1), dev)
        with pytest.raises(bp.BulletproofError, match="differs from the generator set"):
            bp.batch_range_proof_verify_gens(other, gens, torch.zeros(2, dtype=torch.uint8, device=dev))
    finally:
        gens.close()


def test_prefix_tables_reject_busy_and_bad_bits(bp, oracle):
    import torch
    from cudabulletproof_amd import synth
    n = 16
    dev = torch.device("cuda:0")
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a, np.uint64).view(np.int64)).to(dev)
    G, H = oracle.base_points(n, 1), oracle.base_points(n, 2)
    _, h = oracle.gh()
    pipe = bp.VerifyPipeline(4, n, T(G), T(H), T(h))
    with pytest.raises(bp.BulletproofError):
        pipe.prefix_tables(25)
    batch = bp.RangeProofBatch.from_numpy(n, synth.proofs(4, n, seed=3), dev)
    pipe.push(batch, torch.zeros(4, dtype=torch.uint8, device=dev))
    with pytest.raises(bp.BulletproofError):
        pipe.prefix_tables(4)
    pipe.flush()
    pipe.prefix_tables(4)
    pipe.prefix_tables(0)
    pipe.close()


@pytest.mark.parametrize("n,B,K", [(16, 40, 9), (64, 70, 14), (4, 3, 2)])
def test_gens_prover_and_pipeline_same_bits(bp, oracle, n, B, K):
    """A generator set with prefix tables (hipbp_gens_create): the prover on it gives the same
    proofs as without tables (and a sample equals the oracle's prover), and a verify pipeline on
    the same set gives the same verdicts / P / check points as one on the plain generators."""
    import torch
    from cudabulletproof_amd import synth
    dev = torch.device("cuda:0")
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a, np.uint64).view(np.int64)).to(dev)
    G, H = oracle.base_points(n, 1), oracle.base_points(n, 2)
    g, h = oracle.gh()
    rng = np.random.default_rng(n + K)
    values = [np.concatenate([rng.integers(0, 256, max(1, n // 8)).astype(np.uint8),
                              np.zeros(32 - max(1, n // 8), np.uint8)]) for _ in range(B)]
    if n % 8:
        for v in values:
            v[0] &= (1 << n) - 1
    v, gam, sL, sR, rnd, rb = _prove_inputs([300 + p for p in range(B)], values, n)
    Gd, Hd, gd, hd = T(G), T(H), T(g), T(h)
    gens = bp.Generators(n, Gd, Hd, gd, hd, prefix_bits=K)
    args = [T(x) for x in (v, gam, sL, sR, rnd)]
    o0 = bp.batch_generate_range_proof(n, *args, Gd, Hd, gd, hd)
    o1 = bp.batch_generate_range_proof(n, *args, None, None, None, None, gens=gens)
    torch.cuda.synchronize()
    for k in ("V", "A", "S", "T1", "T2", "taux", "mu", "t", "c", "x", "a", "b", "L", "R", "valid"):
        assert torch.equal(o0[k], o1[k]), k
    from oracle.pyoracle import head_fields
    u = lambda t: t.cpu().numpy().view(np.uint64)
    for p in (0, B - 1):
        pr = oracle.generate_range_proof(values[p], *rb[p], n, G, H, g, h)
        if pr is None:   # refused (validate_range_input's byte rule refuses most values at n < 8)
            assert int(o1["valid"][p]) == 0, p
            continue
        hf = head_fields(pr["head"])
        for k in ("V", "A", "S", "T1", "T2", "t", "x"):
            assert np.array_equal(u(o1[k])[p], hf[k]), (p, k)
        assert np.array_equal(u(o1["L"])[p], pr["L"]), p
    batch = bp.RangeProofBatch(n, **{k: o1[k] for k in bp.RangeProofBatch.FIELDS})
    res = []
    for use in (False, True):
        pipe = bp.VerifyPipeline(B, n, Gd, Hd, hd)
        if use:
            pipe.use_gens(gens)
        o = [torch.zeros(B, dtype=torch.uint8, device=dev), torch.zeros(B, 16, dtype=torch.int64, device=dev),
             torch.zeros(B, 16, dtype=torch.int64, device=dev)]
        pipe.push(batch, *o)
        pipe.flush()
        torch.cuda.synchronize()
        res.append([x.cpu() for x in o])
        pipe.close()
    for a, b2 in zip(*res):
        assert torch.equal(a, b2)
    gens.close()


@pytest.mark.gpu
@pytest.mark.parametrize("n,B,K", [(64, 24, 6), (256, 8, 10), (4096, 4, 12)])
def test_gens_inner_product_pipeline_same_bits(bp, oracle, n, B, K):
    """Inner-product mode (cuda_inner_product_verify, bench configs[3]) on a generator set whose g and
    h are both Q: fold round 0 on G/H starts from the prefix tables; verdicts and check points are
    bit-identical to the table-free pipeline."""
    import torch
    from cudabulletproof_amd import synth
    dev = torch.device("cuda:0")
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a, np.uint64).view(np.int64)).to(dev)
    G, H = oracle.base_points(n, 1), oracle.base_points(n, 2)
    _, h = oracle.gh()
    Gd, Hd, Qd = T(G), T(H), T(h)
    arrays = synth.proofs(B, n, seed=70 + K)
    Pg = T(oracle.base_points(B, 9))
    gens = bp.Generators(n, Gd, Hd, Qd, Qd, prefix_bits=K)
    res = []
    for use in (False, True):
        pipe = bp.VerifyPipeline(B, n, Gd, Hd, Qd, range_mode=False)
        if use:
            pipe.use_gens(gens)
        ok = torch.zeros(B, dtype=torch.uint8, device=dev)
        chk = torch.zeros(B, 16, dtype=torch.int64, device=dev)
        pipe.push(bp.RangeProofBatch.from_numpy(n, arrays, dev), ok, None, chk, P_in=Pg)
        pipe.flush()
        torch.cuda.synchronize()
        res.append((ok.cpu(), chk.cpu()))
        pipe.close()
    gens.close()
    assert torch.equal(res[0][0], res[1][0]) and torch.equal(res[0][1], res[1][1])


@pytest.mark.gpu
@pytest.mark.parametrize("n,count,K", [(64, 3, 6), (256, 2, 10), (4096, 2, 12)])
def test_msm_batch_gens_same_bits(bp, oracle, n, count, K):
    """hipbp_msm_batch_gens (canonical MSMs over a generator set's G||H, prefix-table starts) ==
    hipbp_msm_batch over cat(G, H), bit for bit, including zero scalars and scalars with exactly
    K and K - 1 leading zeros; one small case also equals the oracle."""
    import torch
    dev = torch.device("cuda:0")
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a, np.uint64).view(np.int64)).to(dev)
    G, H = oracle.base_points(n, 1), oracle.base_points(n, 2)
    g, h = oracle.gh()
    rng = np.random.default_rng(n + K)
    s = rand_fe(rng, count * 2 * n)
    s[0] = 0
    s[1, :3] = 0
    s[1, 3] = np.uint64(1) << np.uint64(63 - K)          # exactly K leading zeros
    s[2, 3] = (np.uint64(1) << np.uint64(64 - K)) | np.uint64(5)   # K - 1 leading zeros
    Gd, Hd = T(G), T(H)
    gens = bp.Generators(n, Gd, Hd, T(g), T(h), prefix_bits=K)
    sd = T(s)
    r0 = torch.zeros(count, 16, dtype=torch.int64, device=dev)
    r1 = torch.zeros(count, 16, dtype=torch.int64, device=dev)
    bp.msm_batch(r0, sd, torch.cat([Gd, Hd]).contiguous())
    bp.msm_batch_gens(r1, sd, gens)
    torch.cuda.synchronize()
    assert torch.equal(r0, r1)
    if n == 64:
        GH = np.concatenate([G, H])
        assert np.array_equal(r1[0].cpu().numpy().view(np.uint64), oracle.msm_canon(s[:2 * n], GH))
    gens.close()
