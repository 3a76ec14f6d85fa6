"""bench.py's N>1 path (torchrun, one process per rank) rehearsed on one GPU: every rank on cuda:0
with gloo collectives (--rehearse), N = 2, 4, 8.  The sharded MSM (shard roots + all_gather + canonical tree)
and the window-sharded Pippenger (window sums + all_gather + Horner) must give the same points as
the single-rank run, and the line must carry the N-rank fields.  A real (non-rehearsal) N > 1 run
must refuse to measure when its ranks do not sit on N distinct devices or the backend is not RCCL."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SMALL = ["--steps", "2", "--warmup", "1", "--batch", "128", "--msm-log2", "12", "--prefix-bits", "12",
         "--shard-total", "3000", "--no-host", "--no-cpu", "--no-ipa", "--no-prove"]


# rank 0's single-GPU legs (IPA, prover) while the other rank waits at the closing barrier
LEGS = ["--ipa-n", "256", "--ipa-batch", "8", "--ipa-steps", "2", "--prove-batch", "256", "--prove-steps", "1"]


def _line(out):
    return json.loads([l for l in out.splitlines() if l.startswith("{")][-1])


@pytest.fixture(scope="module")
def one_rank_line():
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    one = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + SMALL, capture_output=True, text=True,
                         timeout=600, cwd=ROOT, env=env)
    assert one.returncode == 0, one.stderr[-2000:]
    return _line(one.stdout)


@pytest.mark.gpu
@pytest.mark.parametrize("N", [2, 4, 8])
def test_bench_ranks_rehearsal_matches_one_rank(one_rank_line, N):
    """N = 2, 4, 8 ranks (all on cuda:0, gloo): the shard of configs[4] (shard.shard_bounds(3000, N, r)),
    the sharded canonical MSM and the window-split Pippenger give the one-rank digests."""
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    l1 = one_rank_line
    # no outer launcher: `--gpus N` makes bench.py start the N ranks itself (torch.distributed.run child)
    # N = 8: bench.py's own launcher parent runs the CPU legs (GPU-free, before the spawn) for rank 0's
    # line; N = 4: an outer torchrun (the driver's way) starts the ranks and rank 0 runs them itself
    small = [a for a in SMALL[:-2] if a != "--no-cpu"] + ["--cpu-seconds", "0.5", "--cpu-procs", "2"] \
        if N in (4, 8) else SMALL[:-2]
    outer = []
    if N == 4:
        import socket
        with socket.socket() as so:
            so.bind(("127.0.0.1", 0))
            port = so.getsockname()[1]
        outer = ["-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={N}", "--master-addr", "127.0.0.1",
                 "--master-port", str(port)]
    two = subprocess.run([sys.executable] + outer + [os.path.join(ROOT, "bench.py"), "--gpus", str(N), "--rehearse"]
                         + small + LEGS, capture_output=True, text=True, timeout=900, cwd=ROOT, env=env)
    assert two.returncode == 0, two.stderr[-2000:]
    l2 = _line(two.stdout)
    assert l1["n_gpus"] == 1 and l2["n_gpus"] == N
    # the line proves who ran: the torch.distributed world, one entry per rank, each rank's own batches
    assert l1["world_size"] == 1 and l2["world_size"] == N and l2["backend"] == "gloo"
    assert [r["rank"] for r in l2["ranks"]] == list(range(N)) and len(l1["ranks"]) == 1
    assert l2["ranks"][0]["verdicts_sha256"] == l1["ranks"][0]["verdicts_sha256"]   # rank 0's seeds whatever N
    assert len({r["verdicts_sha256"] for r in l2["ranks"]}) == N                    # distinct batches per rank
    assert all(r["pci"] and r["proofs"] == 4 * 128 for r in l2["ranks"])
    assert l2["msm"]["scaling"] == "strong" and l2["scaling"] == "weak"
    assert l1["msm"]["result_sha256"] == l2["msm"]["result_sha256"]
    # Pippenger with its windows split over the N ranks == the single-GPU Pippenger
    ps = l2["msm"]["pippenger_sharded"]
    assert ps["scaling"] == "strong" and ps["result_sha256"] == l1["msm"]["pippenger"]["result_sha256"]
    # configs[4]: the same proof set sharded over 1 or N ranks -> the same verdicts on every rank
    s1, s2 = l1["sharded_2p16"], l2["sharded_2p16"]
    assert s1["proofs"] == s2["proofs"] == 3000 and s2["scaling"] == "strong"
    assert s1["passes"] == s2["passes"] > 0 and s1["verdicts_sha256"] == s2["verdicts_sha256"]
    assert s1["same_verdicts_every_pass"] and s2["same_verdicts_every_pass"] and s2["passes_timed"] == 5
    # the repeated timed regions of the headline ran on every rank (max over ranks per region)
    assert l1["repeats"]["n"] == l2["repeats"]["n"] == 5
    assert l2["config"]["passes_in_warmup_batch"] >= l1["config"]["passes_in_warmup_batch"]
    assert l2["ipa"]["n_gpus"] == 1 and l2["prove"]["n_gpus"] == 1 and l2["prove"]["valid"] == 256
    assert l1["launcher"] is None
    if N == 4:
        assert l2["launcher"] is None   # started by the outer launcher
    else:
        assert l2["launcher"]["hip_mapped_before_spawn"] == []
    if N in (4, 8):   # the N-rank line carries the CPU baseline (parent or rank 0 timed it)
        assert l2["cpu_baseline"] is not None and l2["cpu_baseline"]["value"] > 0
        assert l2["configs0"] is not None


@pytest.mark.gpu
def test_bench_more_gpus_than_visible_fails():
    """`bench.py --gpus 2` on a one-GPU box must fail, not print a one-GPU line labelled N = 2."""
    import torch
    if torch.cuda.device_count() >= 2:
        pytest.skip("more than one GPU visible")
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"] + SMALL, capture_output=True,
                       text=True, timeout=300, cwd=ROOT)
    assert p.returncode == 3 and "needs 2 GPUs" in p.stderr and not p.stdout.strip()


@pytest.mark.gpu
def test_launcher_gpu_count_matches_hip():
    """bench.py's launcher counts GPUs without the HIP runtime (KFD topology + render nodes +
    visible-device lists); on a GPU box that count must equal what the ranks' HIP runtime sees."""
    import torch
    sys.path.insert(0, ROOT)
    import bench
    assert bench.kfd_gpu_count() == torch.cuda.device_count()
