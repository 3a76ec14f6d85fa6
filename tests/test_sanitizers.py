"""SURVEY §5 (race detection / sanitizers): the CPU restatement (oracle/bp_oracle.c) and the
product's field arithmetic in its host pass (csrc/fe25519_dev.h via tests/host_arith_check.hip)
built with AddressSanitizer + UndefinedBehaviourSanitizer (host code only) and run: no reports,
and the host pass still matches the oracle bit for bit.  GPU kernels are deterministic by
construction (fixed reduction orders, no atomics on point values) and are checked run-to-run by
the -m gpu tests."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SAN = ["-fsanitize=address,undefined", "-fno-sanitize-recover=all"]


@pytest.mark.skipif(shutil.which("gcc") is None, reason="gcc not available")
def test_oracle_under_asan_ubsan(tmp_path):
    exe = tmp_path / "drv"
    subprocess.run(["gcc", "-O1", "-g", "-std=c11"] + SAN + ["-o", str(exe),
                    os.path.join(ROOT, "tests", "sanitize_driver.c"), os.path.join(ROOT, "oracle", "bp_oracle.c")],
                   check=True, capture_output=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    assert r.stdout.startswith("ok "), r.stdout
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr, r.stderr[-3000:]


@pytest.mark.skipif(shutil.which("hipcc") is None, reason="hipcc not available")
def test_product_host_pass_under_asan_ubsan(tmp_path):
    clang = "/opt/rocm/llvm/bin/clang"
    if not os.path.exists(clang):
        pytest.skip("ROCm clang not available")
    orc = tmp_path / "orc.o"
    hac = tmp_path / "hac.o"
    exe = tmp_path / "hac"
    subprocess.run([clang, "-O1", "-g", "-std=c11"] + SAN + ["-c", os.path.join(ROOT, "oracle", "bp_oracle.c"),
                    "-o", str(orc)], check=True, capture_output=True)
    host_san = []
    for f in SAN:   # host code only: each sanitizer flag right after -Xarch_host
        host_san += ["-Xarch_host", f]
    subprocess.run(["hipcc", "-O1", "-g", "-std=c++17", "--cuda-host-only", "-x", "hip",
                    os.path.join(ROOT, "tests", "host_arith_check.hip"), "-c", "-o", str(hac)] + host_san,
                   check=True, capture_output=True)
    subprocess.run(["hipcc", str(hac), str(orc), "-o", str(exe)] + host_san, check=True, capture_output=True)
    r = subprocess.run([str(exe), "30000", "11"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    counts = dict(line.split() for line in r.stdout.split("\n") if line.strip())
    assert set(counts) == {"add", "sub", "mul", "sq", "canon", "fold", "invert"}, r.stdout
    assert all(v == "0" for v in counts.values()), r.stdout
