"""Synthetic-input generator (bench inputs): shapes, determinism, and that its generator
X/Y limbs equal the reference-derived ones (complete_bulletproof_test.cu:33-109)."""
import numpy as np

from cudabulletproof_amd import synth


def test_proof_batch_shapes_and_determinism():
    a = synth.proofs(8, 64, seed=3)
    b = synth.proofs(8, 64, seed=3)
    assert a["L"].shape == (8, 6, 16) and a["a"].shape == (8, 1, 4) and a["V"].shape == (8, 16)
    for k in a:
        assert np.array_equal(a[k], b[k])
    assert (a["b"][:, 0, 0] == 1).all() and np.array_equal(a["a"][:, 0], a["c"])
    assert len({a["V"][i].tobytes() for i in range(8)}) == 8     # distinct proofs


def test_generator_xy_match_reference_fixture(golden):
    d = golden("proofs_n64")
    G = synth.base_points_xy(64, 1)
    assert np.array_equal(G[:, :12], d["G"][:, :12])
    g, h = synth.gh_xy()
    assert np.array_equal(g[:12], d["g"][:12]) and np.array_equal(h[:12], d["h"][:12])
