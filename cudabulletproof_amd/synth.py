"""Deterministic synthetic inputs for the batched verify (bench.py) and the MSM microbench.

Proof-shaped data only: random 255-bit coordinates and scalars from a seeded numpy
generator, laid out in the flat wire format of include/cudabulletproof_hip.h.  Proofs
follow the shape the reference prover emits after fix_inner_product_proof
(bulletproof_range_proof.cu:198-235): a = [t], b = [1], c = t, so the <a,b> = c check
(crv:146-158) passes and every verify runs the full fold.  Verify cost does not depend
on whether a proof is "valid" beyond that check.

Generator points follow complete_bulletproof_test.cu:33-109 (SHA-256 derived X, Y,
Z = 1); their T = X*Y is computed on the GPU by the engine's own field multiply.
"""
import hashlib

import numpy as np

MASK63 = np.uint64(0x7FFFFFFFFFFFFFFF)


def _le_limbs(b32):
    return np.frombuffer(b32, dtype="<u8").astype(np.uint64)


def base_points_xy(n, seed_byte, lo=0):
    """X, Y limbs of generate_deterministic_base_points (complete_bulletproof_test.cu:33-63),
    points lo .. lo+n-1."""
    seed = bytes([seed_byte]) + bytes(31)
    xs = bytearray()
    ys = bytearray()
    for i in range(lo, lo + n):
        x = hashlib.sha256(seed + int(i).to_bytes(4, "big")).digest()
        xs += x
        ys += hashlib.sha256(x).digest()
    pts = np.zeros((n, 16), np.uint64)
    pts[:, 0:4] = np.frombuffer(bytes(xs), dtype="<u8").reshape(n, 4)
    pts[:, 4:8] = np.frombuffer(bytes(ys), dtype="<u8").reshape(n, 4)
    pts[:, 8] = 1
    return pts


def gh_xy():
    """X limbs of g, h (complete_bulletproof_test.cu:84-109): X = SHA256({3}/{4} || 0^31), Y = Z = 1."""
    out = []
    for sb in (3, 4):
        p = np.zeros(16, np.uint64)
        p[0:4] = _le_limbs(hashlib.sha256(bytes([sb]) + bytes(31)).digest())
        p[4] = 1
        p[8] = 1
        out.append(p)
    return out


def fill_T(points, device):
    """T = X*Y with the engine's fe25519_mul (in place on a numpy (k,16) array)."""
    import torch
    from . import field_op
    pts = np.ascontiguousarray(points).reshape(-1, 16)
    X = torch.from_numpy(np.ascontiguousarray(pts[:, 0:4]).view(np.int64)).to(device)
    Y = torch.from_numpy(np.ascontiguousarray(pts[:, 4:8]).view(np.int64)).to(device)
    T = torch.empty_like(X)
    field_op("mul", T, X, Y)
    torch.cuda.synchronize(device)
    pts[:, 12:16] = T.cpu().numpy().view(np.uint64)
    return pts


def generators(n, device):
    """G, H (n,16), g, h (16,) as numpy, T filled on the GPU."""
    G = base_points_xy(n, 1)
    H = base_points_xy(n, 2)
    g, h = gh_xy()
    allp = np.concatenate([G, H, g[None], h[None]])
    allp = fill_T(allp, device)
    return allp[:n], allp[n:2 * n], allp[2 * n], allp[2 * n + 1]


def _rand_fe(rng, shape):
    v = rng.integers(0, 2**64, size=shape + (4,), dtype=np.uint64)
    v[..., 3] &= MASK63
    return v


def _rand_pt(rng, shape):
    p = np.zeros(shape + (16,), np.uint64)
    p[..., 0:4] = _rand_fe(rng, shape)
    p[..., 4:8] = _rand_fe(rng, shape)
    p[..., 8] = 1
    p[..., 12:16] = _rand_fe(rng, shape)   # T is not read by the verify path
    return p


def proofs(count, n, seed=1):
    """Synthetic proof batch (numpy dict in the flat wire format)."""
    rng = np.random.default_rng(seed)
    Lr = int(n).bit_length() - 1
    t = _rand_fe(rng, (count,))
    t[:, 3] &= np.uint64(0x3FFFFFFFFFFFFFFF)   # t < p, so <[t],[1]> = t canonically
    one = np.zeros((count, 1, 4), np.uint64)
    one[..., 0] = 1
    return dict(
        V=_rand_pt(rng, (count,)), A=_rand_pt(rng, (count,)), S=_rand_pt(rng, (count,)),
        T1=_rand_pt(rng, (count,)), T2=_rand_pt(rng, (count,)), t=t, a=t[:, None, :].copy(), b=one,
        c=t.copy(), x=_rand_fe(rng, (count,)), L=_rand_pt(rng, (count, Lr)), R=_rand_pt(rng, (count, Lr)))


def msm_config3(lo, hi, device):
    """SURVEY §8(d) config 3 (BASELINE configs[2]), rows lo..hi-1 of the 2^20-point MSM input:
    points = base points with seed {5} (T = X*Y on the GPU), scalars_i = SHA256("msm-s" || i_le32)
    with byte 31 &= 0x7F.  tests/golden/msm_2p20.json holds the expected result for all 2^20."""
    sc = bytearray()
    for i in range(lo, hi):
        sc += hashlib.sha256(b"msm-s" + int(i).to_bytes(4, "little")).digest()
    s = np.frombuffer(bytes(sc), dtype="<u8").reshape(hi - lo, 4).copy()
    s[:, 3] &= MASK63
    return s, fill_T(base_points_xy(hi - lo, 5, lo), device)


def msm_inputs(n, seed=5):
    """MSM microbench inputs: points = random (X, Y, Z=1, T), scalars = 255-bit."""
    rng = np.random.default_rng(seed)
    return _rand_fe(rng, (n,)), _rand_pt(rng, (n,))


def _rand_scalar(rng, shape):
    """Random scalars as generate_random_scalar (rp.cu:153-159) shapes them: byte 0 &= 0xF8,
    byte 31 &= 0x7F then |= 0x40 — as LE u64 limbs."""
    v = rng.integers(0, 2**64, size=shape + (4,), dtype=np.uint64)
    v[..., 0] &= np.uint64(0xFFFFFFFFFFFFFFF8)
    v[..., 3] = (v[..., 3] & np.uint64(0x7FFFFFFFFFFFFFFF)) | np.uint64(0x4000000000000000)
    return v


def prove_inputs(count, n, seed=11):
    """Prover inputs (hipbp_prove_input layout): values uniform in [0, 2^n), random scalars."""
    rng = np.random.default_rng(seed)
    v = np.zeros((count, 4), np.uint64)
    if n >= 64:
        v[:, 0] = rng.integers(0, 2**64, size=count, dtype=np.uint64)
        for k in range(1, n // 64):
            v[:, k] = rng.integers(0, 2**64, size=count, dtype=np.uint64)
    else:
        v[:, 0] = rng.integers(0, 2**n, size=count, dtype=np.uint64)
    return dict(v=v, gamma=_rand_scalar(rng, (count,)), sL=_rand_scalar(rng, (count, n)),
                sR=_rand_scalar(rng, (count, n)), rnd=_rand_scalar(rng, (count, 4)))
