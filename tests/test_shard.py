"""Multi-GPU sharding (cudabulletproof_amd/shard.py).

CPU tests: the shard plans, the canonical-tree decomposition the multi-GPU MSM relies on
(checked with the oracle), and the torch.distributed logic at world_size 2 on gloo with
the oracle standing in for the per-rank HIP kernels.  GPU tests: hipbp_point_tree and the
sharded MSM (ranks emulated in one process) against the single-GPU MSM, bit for bit.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from cudabulletproof_amd import shard


def test_shard_bounds_cover_everything():
    for total in (0, 1, 7, 1024, 65536, 65537):
        for world in (1, 2, 3, 8):
            spans = [shard.shard_bounds(total, world, r) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == total
            assert all(spans[i][1] == spans[i + 1][0] for i in range(world - 1))
            sizes = [h - l for l, h in spans]
            assert max(sizes) - min(sizes) <= 1


@pytest.mark.parametrize("n", [1, 2, 5, 64, 100, 1 << 20, (1 << 20) + 3])
@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_msm_plan(n, world):
    m, K = shard.msm_shard_plan(n, world)
    assert m & (m - 1) == 0 and m * world >= n and 1 <= K <= world and (K - 1) * m < n <= K * m
    spans = [shard.msm_shard_bounds(n, world, r) for r in range(world)]
    assert spans[0][0] == 0 and spans[K - 1][1] == n
    assert all(l == h for l, h in spans[K:])


def _np(t):
    return t.detach().cpu().numpy().view(np.uint64)


def _oracle_fns(O):
    def local_msm(s, P):
        return torch.from_numpy(O.msm_canon(_np(s), _np(P)).view(np.int64))

    def tree(P):
        return torch.from_numpy(O.point_tree(_np(P)).view(np.int64))
    return local_msm, tree


def _inputs(n, seed):
    from cudabulletproof_amd import synth
    s, P = synth.msm_inputs(n, seed=seed)
    return s, P


@pytest.mark.parametrize("n", [1, 3, 16, 37, 100])
@pytest.mark.parametrize("world", [2, 3, 4, 8])
def test_tree_decomposition_is_bit_exact(oracle, n, world):
    """Shard roots + canonical tree over them == the single-GPU canonical-tree MSM."""
    s, P = _inputs(n, seed=11)
    m, K = shard.msm_shard_plan(n, world)
    roots = np.stack([oracle.msm_canon(s[lo:hi], P[lo:hi])
                      for lo, hi in (shard.msm_shard_bounds(n, world, r) for r in range(K))])
    assert np.array_equal(oracle.point_tree(roots), oracle.msm_canon(s, P))


def _free_port():
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def _worker(rank, world, port, n, total, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from oracle import pyoracle
        O = pyoracle.Oracle()
        s, P = _inputs(n, seed=3)
        lo, hi = shard.msm_shard_bounds(n, world, rank)
        local_msm, tree = _oracle_fns(O)
        r = shard.sharded_msm(torch.from_numpy(s[lo:hi].view(np.int64)), torch.from_numpy(P[lo:hi].view(np.int64)),
                              n, local_msm=local_msm, tree=tree)
        vlo, vhi = shard.shard_bounds(total, world, rank)
        ok = torch.from_numpy((np.arange(vlo, vhi) % 3 == 0).astype(np.uint8))
        allok = shard.gather_verdicts(ok, total)
        passes = torch.tensor([int(ok.sum())], dtype=torch.int64)
        dist.all_reduce(passes)
        q.put((rank, _np(r).copy(), allok.numpy().copy(), int(passes.item())))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,n,total", [(2, 37, 11), (2, 64, 1024), (3, 5, 7)])
def test_gloo_sharded_msm_and_verdicts(oracle, world, n, total):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n, total, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    s, P = _inputs(n, seed=3)
    want = oracle.msm_canon(s, P)
    want_ok = (np.arange(total) % 3 == 0).astype(np.uint8)
    for rank, r, allok, passes in res:
        assert np.array_equal(r, want), f"rank {rank}"
        assert np.array_equal(allok, want_ok) and passes == int(want_ok.sum())


@pytest.mark.gpu
@pytest.mark.parametrize("n", [1, 2, 3, 255, 256, 257, 1000, 70000])
def test_point_tree_matches_oracle(bp, oracle, n):
    rng = np.random.default_rng(n)
    pts = np.zeros((n, 16), np.uint64)
    pts[:] = rng.integers(0, 2**64, size=(n, 16), dtype=np.uint64)
    pts[:, 3::4] &= np.uint64(0x7FFFFFFFFFFFFFFF)
    dev = torch.device("cuda:0")
    out = torch.zeros(16, dtype=torch.int64, device=dev)
    bp.point_tree(out, torch.from_numpy(pts.view(np.int64)).to(dev))
    torch.cuda.synchronize()
    assert np.array_equal(_np(out), oracle.point_tree(pts))


@pytest.mark.gpu
@pytest.mark.parametrize("n,world", [(100, 2), (4096, 8), (5000, 3)])
def test_sharded_msm_emulated_ranks_match_single_gpu(bp, n, world):
    """The shard roots + point_tree combine (what sharded_msm does across ranks) on one GPU."""
    dev = torch.device("cuda:0")
    s, P = _inputs(n, seed=8)
    sd, Pd = torch.from_numpy(s.view(np.int64)).to(dev), torch.from_numpy(P.view(np.int64)).to(dev)
    full = torch.zeros(16, dtype=torch.int64, device=dev)
    bp.msm(full, sd, Pd)
    m, K = shard.msm_shard_plan(n, world)
    roots = []
    for r in range(K):
        lo, hi = shard.msm_shard_bounds(n, world, r)
        roots.append(shard._hip_msm(sd[lo:hi], Pd[lo:hi]))
    comb = shard._hip_tree(torch.stack(roots))
    torch.cuda.synchronize()
    assert np.array_equal(_np(comb), _np(full))


# ---- window-sharded Pippenger (shard.sharded_msm_pippenger) ----

@pytest.mark.parametrize("c", [4, 5, 8, 12])
def test_pippenger_window_bounds_cover_every_window(c):
    W = (256 + c - 1) // c
    for world in (1, 2, 3, 8, W + 3):
        spans = [shard.pippenger_window_bounds(c, world, r) for r in range(world)]
        assert spans[0][0] == 0 and spans[-1][1] == W
        assert all(spans[i][1] == spans[i + 1][0] for i in range(world - 1))


@pytest.mark.parametrize("n,c,splits", [(1, 4, [0, 64]), (37, 5, [0, 7, 30, 52]), (300, 8, [0, 1, 31, 32]),
                                        (1000, 12, [0, 5, 11, 22])])
def test_pippenger_windows_then_horner_is_the_msm(oracle, n, c, splits):
    """Window sums formed in pieces + the Horner == orc_msm_pippenger (the split is exact)."""
    s, P = _inputs(n, seed=21)
    Sw = np.concatenate([oracle.pippenger_windows(s, P, c, a, b) for a, b in zip(splits, splits[1:])])
    assert np.array_equal(oracle.pippenger_horner(Sw, c), oracle.msm_pippenger(s, P, c))


def _oracle_pip_fns(O):
    def windows(sc, P, w0, w1, c):
        return torch.from_numpy(O.pippenger_windows(_np(sc), _np(P), c, w0, w1).view(np.int64))

    def horner(Sw, c):
        return torch.from_numpy(O.pippenger_horner(_np(Sw), c).view(np.int64))
    return windows, horner


def _pip_worker(rank, world, port, n, c, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from oracle import pyoracle
        O = pyoracle.Oracle()
        s, P = _inputs(n, seed=4)
        windows, horner = _oracle_pip_fns(O)
        r = shard.sharded_msm_pippenger(torch.from_numpy(s.view(np.int64)), torch.from_numpy(P.view(np.int64)), c,
                                        windows=windows, horner=horner)
        q.put((rank, _np(r).copy()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,n,c", [(2, 200, 8), (3, 64, 12), (2, 33, 5)])
def test_gloo_sharded_pippenger(oracle, world, n, c):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_pip_worker, args=(r, world, port, n, c, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    s, P = _inputs(n, seed=4)
    want = oracle.msm_pippenger(s, P, c)
    for rank, r in res:
        assert np.array_equal(r, want), f"rank {rank}"


@pytest.mark.gpu
@pytest.mark.parametrize("n,c,world", [(1, 12, 2), (1000, 8, 3), (5000, 12, 8), (70001, 12, 4), (4096, 5, 8)])
def test_pippenger_windows_emulated_ranks_match_single_gpu(bp, oracle, n, c, world):
    """Each emulated rank's window range (hipbp_msm_pippenger_windows) + one Horner launch ==
    hipbp_msm_pippenger, and both == the oracle (small n)."""
    dev = torch.device("cuda:0")
    s, P = _inputs(n, seed=12)
    sd, Pd = torch.from_numpy(s.view(np.int64)).to(dev), torch.from_numpy(P.view(np.int64)).to(dev)
    full = torch.zeros(16, dtype=torch.int64, device=dev)
    bp.msm_pippenger(full, sd, Pd, c)
    W = bp.pippenger_num_windows(c)
    Sw = torch.zeros(W, 16, dtype=torch.int64, device=dev)
    for r in range(world):
        w0, w1 = shard.pippenger_window_bounds(c, world, r)
        bp.msm_pippenger_windows(Sw, sd, Pd, w0, w1, c)
    out = torch.zeros(16, dtype=torch.int64, device=dev)
    bp.msm_pippenger_horner(out, Sw, c)
    one = shard.sharded_msm_pippenger(sd, Pd, c)   # world 1: all windows in one call
    torch.cuda.synchronize()
    assert np.array_equal(_np(out), _np(full)) and np.array_equal(_np(one), _np(full))
    if n <= 5000:
        assert np.array_equal(_np(out), oracle.msm_pippenger(s, P, c))
        assert np.array_equal(_np(Sw)[2:4], oracle.pippenger_windows(s, P, c, 2, 4))


@pytest.mark.gpu
def test_pippenger_windows_argument_errors(bp):
    dev = torch.device("cuda:0")
    s, P = _inputs(8, seed=1)
    sd, Pd = torch.from_numpy(s.view(np.int64)).to(dev), torch.from_numpy(P.view(np.int64)).to(dev)
    Sw = torch.zeros(22, 16, dtype=torch.int64, device=dev)
    for w0, w1 in ((-1, 3), (3, 23), (5, 4)):
        with pytest.raises(bp.BulletproofError):
            bp.msm_pippenger_windows(Sw, sd, Pd, w0, w1, 12)
    with pytest.raises(bp.BulletproofError):
        bp.msm_pippenger_windows(Sw, sd, Pd, 0, 3, 13)
    with pytest.raises(bp.BulletproofError):
        bp.msm_pippenger_horner(torch.zeros(16, dtype=torch.int64, device=dev), Sw[:21], 12)
    bp.msm_pippenger_windows(Sw, sd, Pd, 4, 4, 12)   # empty range: nothing written
    torch.cuda.synchronize()
    assert int(Sw.abs().sum().item()) == 0
