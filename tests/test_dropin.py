"""Drop-in check: the reference's own test driver (complete_bulletproof_test.cu) and host code
(bulletproof_range_proof.cu, ...), compiled unchanged by oracle/build_ref.sh and linked against
libcudabulletproof_hip.so in place of the CUDA objects.  Its RNG is the
deterministic stream of oracle/ref/det_rand.c, so its 16-bit proof is tests/golden proofs_n16[0]."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "oracle", "_ref", "complete_bulletproof_test_hip")


def test_dropin_binary_links_our_library():
    if not os.path.exists(BIN):
        pytest.skip("oracle/_ref not built (needs /root/reference at build time)")
    out = subprocess.check_output(["ldd", BIN], text=True)
    assert "libcudabulletproof_hip.so" in out


@pytest.mark.gpu
def test_reference_driver_runs_on_our_library():
    if not os.path.exists(BIN):
        pytest.skip("oracle/_ref not built")
    env = dict(os.environ, BP_RAND_SEED="1")
    # line-buffered stdout: the driver ends in undefined behaviour of its own
    # (complete_bulletproof_test.cu:305 frees the never-initialised ip_proof of the rejected
    # out-of-range proof), which can crash it after everything below is printed:
    # SIGSEGV, or SIGABRT from glibc's "free(): invalid pointer", depending on stack contents.
    p = subprocess.run(["stdbuf", "-oL", BIN], capture_output=True, text=True, timeout=300, env=env)
    out = p.stdout
    # complete_bulletproof_test.cu:179-191 / :247-255
    assert "CUDA Verification result: SUCCESS" in out, out[-3000:]
    assert "CPU Verification result: SUCCESS" in out, out[-3000:]
    assert "FAILED (CORRECT)" in out, out[-3000:]
    assert "CUDA FIELD OPERATIONS BENCHMARK" in out
    assert "CUDA field squaring:" in out           # the last GPU call the driver makes
    assert p.returncode in (0, -6, -11, 134, 139), p.returncode
