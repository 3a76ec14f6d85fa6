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
    monkeypatch.setattr(subprocess, "call", lambda cmd, env=None: seen.update(cmd=cmd, env=env) or 0)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "4", "--rehearse", "--steps", "3"])
    a = argparse.Namespace(gpus=4, rehearse=True, no_cpu=True)
    assert bench.rank_launch(a) == 0
    cmd = seen["cmd"]
    # the CPU legs' hand-over file is named to the ranks and removed after them
    assert seen["env"]["BENCH_CPU_LEGS"] and not os.path.exists(seen["env"]["BENCH_CPU_LEGS"])
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


def _kfd_node(root, name, simd, minor):
    d = os.path.join(root, name)
    os.makedirs(d)
    with open(os.path.join(d, "properties"), "w") as f:
        f.write(f"cpu_cores_count {0 if simd else 64}\nsimd_count {simd}\n")
        if minor is not None:
            f.write(f"drm_render_minor {minor}\n")


def test_kfd_gpu_count(tmp_path):
    """The launcher counts GPUs from the KFD topology without the HIP runtime: nodes with SIMDs whose
    render node exists in this container, capped by the visible-device lists."""
    sysfs, dri = str(tmp_path / "nodes"), str(tmp_path / "dri")
    os.makedirs(dri)
    _kfd_node(sysfs, "0", 0, None)           # a CPU node
    for i, minor in enumerate((128, 136, 144)):
        _kfd_node(sysfs, str(i + 1), 1024, minor)
    for minor in (128, 136):                 # the third GPU is not passed to this container
        open(os.path.join(dri, f"renderD{minor}"), "w").close()
    assert bench.kfd_gpu_count(sysfs, dri, env={}) == 2
    assert bench.kfd_gpu_count(sysfs, dri, env={"HIP_VISIBLE_DEVICES": "1"}) == 1
    assert bench.kfd_gpu_count(sysfs, dri, env={"ROCR_VISIBLE_DEVICES": "0,1,2,3"}) == 2
    assert bench.kfd_gpu_count(str(tmp_path / "absent"), dri, env={}) is None


def test_hip_mapped_probe_sees_torch():
    """hip_mapped() reads /proc/self/maps: a process that imported torch (a ROCm build) has the HIP runtime
    mapped, a bare interpreter has not — the probe the launcher's HIP-free check relies on."""
    import subprocess
    code = "import sys; sys.path.insert(0, %r); import bench; a = bench.hip_mapped(); import torch; " \
           "print(bool(a), bool(bench.hip_mapped()))" % ROOT
    p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-2000:]
    before, after = p.stdout.split()
    assert before == "False"
    import torch
    if torch.version.hip:
        assert after == "True"


def test_launcher_parent_is_hip_free_and_hands_cpu_legs_to_rank0():
    """`bench.py --gpus N` without a launcher: the parent never maps the HIP runtime up to the spawn,
    and it runs the CPU baseline + configs[0] legs itself, so the N-rank line carries them
    (BENCH_LAUNCH_DRYRUN=1: the parent prints the hand-over instead of spawning)."""
    import json
    p = _run_bench(["--gpus", "2", "--rehearse", "--cpu-seconds", "0.3", "--cpu-procs", "1"],
                   {"BENCH_LAUNCH_DRYRUN": "1"}, timeout=600)
    assert p.returncode == 0, p.stderr[-2000:]
    legs = json.loads(p.stdout.strip().splitlines()[-1])
    assert legs["launcher"]["hip_mapped_before_spawn"] == []
    cpu = legs["cpu_baseline"]
    assert cpu is not None and cpu["value"] > 0 and cpu["cores"] == 1 and cpu["kind"] in ("reference", "port")
    assert not os.path.exists(legs["hand_over"])
