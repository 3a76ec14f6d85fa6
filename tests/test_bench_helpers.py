"""CPU checks of bench.py's accounting (no GPU): SURVEY §8(d)'s algorithmic bytes, the traffic model,
the roofline fields' shape when no PMC run matches, the shard push sizes and the CPU share."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def test_survey_8d_bytes():
    # 944 + 64 n + 256 log2 n per verify (+ 1 B verdict); generators 2 n 128 + 256 per batch
    assert bench.verify_bytes(64) == 6576 + 1
    assert bench.verify_bytes(16) == 2992 + 1
    assert bench.gens_bytes(64) == 16640
    assert bench.alg_bytes("k_terms", 1024, 64) == 1024 * 6577 + 16640
    assert bench.alg_bytes("k_msm_points", 1024, 64) is None


def test_traffic_model_terms():
    m = bench.traffic_model(1024, 64, 22)
    assert m["terms_written_and_read"] == 1024 * bench.sm_per_verify(64) * 288
    assert m["prefix_table_gathers"] == 1024 * 258 * 128
    assert m["msm_lane_trees"] == 1024 * 2 * 63 * 384
    assert bench.traffic_model(1024, 64, 0)["prefix_table_gathers"] == 0
    assert bench.sm_per_verify(64) == 384   # 2n MSM terms + 4 (n/2 + ... + 1) fold terms + t h, c Q, a0 G', b0 H'


def test_rooflines_without_matching_pmc(monkeypatch):
    monkeypatch.setattr(bench, "pmc", lambda *a, **k: None)
    r, v = bench.rooflines("k_terms", 1024, 64, 20, 20, 9.0, 0.108, {"k_terms": 180.0},
                           {"batch_per_gpu": 1024, "n": 64, "prefix_bits": 22, "pipelines": 2}, 2)
    per = 1024 * 6577 + 16640
    assert r["alg_bytes_per_launch"] == per and r["alg_bytes_per_step"] == per
    # the headline frac is driver-consistent: bytes per step / (wall time / steps), 20 steps in 0.108 s
    assert abs(r["achieved"] - per * 20 / 0.108 / 1e9) < 1e-9
    assert abs(r["frac"] - r["achieved"] / bench.HBM_PEAK_GBS) < 1e-15
    # the overlapped per-launch figure only beside it
    assert abs(r["per_launch_overlapped"]["achieved"] - per / 9e-3 / 1e9) < 1e-9
    assert r["frac"] < 1e-3 and r["traffic"] is None and r["traffic_over_alg"] is None
    assert v["frac"] is None and v["achieved_aggregate"] is None


def test_shard_push_batch():
    a = argparse.Namespace(shard_batch=0, batch=1024)
    assert bench.shard_push_batch(a, 8192, 2) == 4096     # N = 8: one push per pipeline
    assert bench.shard_push_batch(a, 65536, 2) == 4096    # N = 1: capped at 4096
    assert bench.shard_push_batch(a, 2048, 2) == 1024
    a.shard_batch = 512
    assert bench.shard_push_batch(a, 8192, 2) == 512


def test_cpu_share(monkeypatch):
    monkeypatch.setenv("OMP_NUM_THREADS", "3")
    nproc, aff, used = bench.cpu_share()
    assert nproc >= aff >= 1 and used == min(aff, 3)
    monkeypatch.delenv("OMP_NUM_THREADS")
    assert bench.cpu_share()[2] == aff


def _run_bench(args, env_extra=None, timeout=240):
    import subprocess
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, capture_output=True, text=True,
                          timeout=timeout, env=env, cwd=ROOT)


def test_gpus_flag_mismatch_with_launcher_world_fails():
    # under a launcher the world must be the --gpus N asked for (no silent 1-rank line)
    p = _run_bench(["--gpus", "8"], {"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert p.returncode == 2 and "WORLD_SIZE=1" in p.stderr


def test_gpus_flag_more_than_visible_fails(monkeypatch):
    # --gpus 2 with fewer visible GPUs (none in this container): an error, not an N = 1 line
    p = _run_bench(["--gpus", "2"])
    assert p.returncode == 3 and "needs 2 GPUs" in p.stderr and not p.stdout.strip()


def test_rank_launch_command(monkeypatch):
    # --gpus N without a launcher: torch.distributed.run --nproc-per-node N on bench.py itself, as a child
    import subprocess
    seen = {}
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setattr(subprocess, "call", lambda cmd: seen.setdefault("cmd", cmd) and 0)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "4", "--rehearse", "--steps", "3"])
    a = argparse.Namespace(gpus=4, rehearse=True)
    assert bench.rank_launch(a) == 0
    cmd = seen["cmd"]
    assert cmd[1:4] == ["-m", "torch.distributed.run", "--nnodes=1"] and "--nproc-per-node=4" in cmd
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[-5:] == ["--gpus", "4", "--rehearse", "--steps", "3"] and cmd[-6].endswith("bench.py")
    assert bench.rank_launch(argparse.Namespace(gpus=1, rehearse=False)) is None


def _distinct_worker(rank, world, port, pcis, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    bench.device_pci = lambda dev: pcis[rank]
    try:
        bench.require_distinct_devices(None, world, rank)
        q.put((rank, "ran"))
        dist.destroy_process_group()
    except SystemExit as e:
        q.put((rank, f"exit {e.code}"))


def test_measured_multirank_run_needs_distinct_devices_over_rccl():
    """A non-rehearsal N-rank bench refuses (exit 4 on every rank, before any leg) when its ranks
    share a device or the backend is not RCCL: here gloo ranks on two distinct and on one shared
    PCI address — both refused, since gloo is not 'nccl'."""
    import multiprocessing as mp
    import socket
    for pcis in (["0000:05:00.0", "0000:15:00.0"], ["0000:05:00.0", "0000:05:00.0"]):
        with socket.socket() as so:
            so.bind(("127.0.0.1", 0))
            port = so.getsockname()[1]
        ctx = mp.get_context("spawn")
        q = ctx.Queue()
        procs = [ctx.Process(target=_distinct_worker, args=(r, 2, port, pcis, q)) for r in range(2)]
        for p in procs:
            p.start()
        res = dict(q.get(timeout=120) for _ in range(2))
        for p in procs:
            p.join(timeout=60)
        assert res == {0: "exit 4", 1: "exit 4"}, res
