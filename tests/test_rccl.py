"""The RCCL side of the N > 1 path on the one GPU a box has.

RCCL refuses two ranks on one device, so the multi-rank logic is covered on gloo
(tests/test_shard.py, tests/test_bench_multirank.py).  This runs the collectives bench.py issues
at N > 1 through the "nccl" backend (= RCCL) in a one-rank group on cuda:0, in a spawned process:
init with device_id, barrier, all_reduce MAX (the timed regions) and SUM (pass counts),
all_gather of the verdict bytes (shard.gather_verdicts) and of the canonical-MSM shard roots
(shard.sharded_msm's gather, fed the HIP MSM's root), each checked against its expected value.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp


def _free_port():
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def _worker(port, q):
    import torch.distributed as dist

    import cudabulletproof_amd as bp
    import cudabulletproof_amd.synth  # noqa: F401  (bp.synth)
    from cudabulletproof_amd import shard
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    try:
        out = {"backend": dist.get_backend()}
        dist.barrier()
        t = torch.tensor([0.25, 1.5], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        out["max"] = t.tolist()
        c = torch.tensor([913], dtype=torch.int64, device=dev)
        dist.all_reduce(c, op=dist.ReduceOp.SUM)
        out["sum"] = int(c.item())
        ok = (torch.arange(3000, device=dev) % 3 == 0).to(torch.uint8)
        out["verdicts"] = shard.gather_verdicts(ok, 3000).cpu().numpy().tobytes() == ok.cpu().numpy().tobytes()
        # the sharded MSM's collective: every rank's root gathered, then the fixed-order tree
        sc, pts = bp.synth.msm_inputs(64, seed=7)
        S = torch.from_numpy(np.ascontiguousarray(sc).view(np.int64)).to(dev)
        P = torch.from_numpy(np.ascontiguousarray(pts).view(np.int64)).to(dev)
        root = shard._hip_msm(S, P)
        parts = [torch.empty(16, dtype=torch.int64, device=dev)]
        dist.all_gather(parts, root.contiguous())
        out["msm_gather"] = bool(torch.equal(parts[0], root)) and bool((root != 0).any())
        dist.barrier()
        torch.cuda.synchronize()
        q.put(out)
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
def test_rccl_collectives_one_rank():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_worker, args=(_free_port(), q))
    p.start()
    try:
        out = q.get(timeout=120)
    finally:
        p.join(timeout=60)
        if p.is_alive():
            p.kill()
    assert p.exitcode == 0
    assert out["backend"] == "nccl"
    assert out["max"] == [0.25, 1.5] and out["sum"] == 913 and out["verdicts"]
    assert out["msm_gather"]
