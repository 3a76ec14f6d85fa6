"""The product's field arithmetic (fe25519_dev.h, __host__ __device__) compiled as HOST code
and checked against the oracle on edge-heavy inputs, including the reference's lossy-carry
corner cases (sub borrow dropped when g_i = 2^64-1, fold carry dropped when 19 t_{i+4} + cy
wraps).  The device pass of the same header differs only in the product columns (gfx950 asm),
which the -m gpu parity tests cover."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("hipcc") is None, reason="hipcc not available")
def test_field_ops_host_pass_match_oracle(oracle, tmp_path):
    exe = tmp_path / "hac"
    subprocess.run(["hipcc", "-O2", "-std=c++17", "--cuda-host-only", "-x", "hip",
                    os.path.join(ROOT, "tests", "host_arith_check.hip"), "-o", str(exe),
                    "-L" + os.path.join(ROOT, "oracle"), "-lbp_oracle",
                    "-Wl,-rpath," + os.path.join(ROOT, "oracle")], check=True, capture_output=True)
    r = subprocess.run([str(exe), "200000", "7"], capture_output=True, text=True, timeout=300)
    counts = dict(line.split() for line in r.stdout.split("\n") if line.strip())
    assert set(counts) == {"add", "sub", "mul", "sq", "canon", "fold", "invert"}, r.stdout
    assert all(v == "0" for v in counts.values()), r.stdout
    assert r.returncode == 0


@pytest.mark.skipif(shutil.which("hipcc") is None, reason="hipcc not available")
def test_split_stage0_lane_layout_host_pass(tmp_path):
    """The verify pipeline's stage-0 lane layout (bp_kernels.h, __host__ __device__) compiled as HOST
    code: the split stage 0's two parts (RK_STAGE0 of a deferred batch, RK_MSMT) reach exactly the
    unsplit stage 0's items, each once, with and without a lane order (tests/host_lanes_check.hip)."""
    exe = tmp_path / "hlc"
    subprocess.run(["hipcc", "-O2", "-std=c++17", "--cuda-host-only", "-x", "hip",
                    os.path.join(ROOT, "tests", "host_lanes_check.hip"), "-o", str(exe)], check=True,
                   capture_output=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    cases, fails = (int(x) for x in r.stdout.split("\n")[-2].split())
    assert r.returncode == 0 and fails == 0 and cases == 168, r.stdout[-2000:]
