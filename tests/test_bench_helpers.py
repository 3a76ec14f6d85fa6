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
    assert r["alg_bytes_per_launch"] == per
    assert abs(r["achieved"] - per / 9e-3 / 1e9) < 1e-9
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
