"""Drop-in check: the reference's own test driver (complete_bulletproof_test.cu, main() unchanged) and
host code (bulletproof_range_proof.cu, ...), compiled by oracle/build_ref.sh and linked against
libcudabulletproof_hip.so in place of the CUDA objects.  Its RNG is the
deterministic stream of oracle/ref/det_rand.c, so its 16-bit proof is tests/golden proofs_n16[0].

The driver ends in undefined behaviour of its own: complete_bulletproof_test.cu:305
range_proof_free(&large_proof) frees the ip_proof that generate_range_proof never initialised for
the refused out-of-range value (bulletproof_range_proof.cu:1176-1187 return before range_proof_init,
SURVEY §3.1).  build_ref.sh compiles the driver with -ftrivial-auto-var-init=pattern, so that free
is always free(0xaaaaaaaaaaaaaaaa) and the process always ends in SIGSEGV after all of its output.
The CPU twin (GPU symbols host-emulated over the reference's own device primitives) and an
ASan + UBSan build of it show the cause; the GPU run must end the same way, print the same lines,
and nothing of ours may fail first."""
import os
import re
import signal
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = os.path.join(ROOT, "oracle", "_ref")
BIN = os.path.join(REF, "complete_bulletproof_test_hip")
CPU = os.path.join(REF, "complete_bulletproof_test_cpu")
ASAN = os.path.join(REF, "complete_bulletproof_test_asan")

LAST_LINE = "CUDA field squaring:"   # the last GPU call main() makes (complete_bulletproof_test.cu:291-295)
# lines cuda_range_proof_verify itself prints (the notebook's crv:82-370 debug chatter): the reference
# prints them inside the function this library replaces, which keeps stdout quiet
CRV_BLOCKS = (("========= STARTING CUDA VERIFICATION =========", "CUDA Verification Time:"),
              ("Verifying range proof for out-of-range value with CUDA...",
               "CUDA Verification result for out-of-range value:"))


def _run(path, env_extra=None):
    env = dict(os.environ, BP_RAND_SEED="1", **(env_extra or {}))
    return subprocess.run(["stdbuf", "-oL", path], capture_output=True, text=True, timeout=300, env=env)


def _norm(lines):
    """Timing values vary run to run: every 'N.NNN seconds' and the speedup factor."""
    return [re.sub(r"Speedup: [0-9.]+x", "Speedup: Sx", re.sub(r"[0-9]+\.[0-9]+ seconds", "T seconds", l))
            for l in lines]


def _without_crv(lines):
    out, skip = [], None
    for l in lines:
        if skip is not None:
            if l.startswith(skip):
                skip = None
                out.append(l)
            continue
        out.append(l)
        for a, b in CRV_BLOCKS:
            if l.startswith(a):
                skip = b
    return out


def _cpu_twin_lines():
    p = _run(CPU)
    assert p.returncode == -signal.SIGSEGV, (p.returncode, p.stderr[-2000:])
    return _norm(p.stdout.splitlines()), p.stderr


def test_dropin_binary_links_our_library():
    if not os.path.exists(BIN):
        pytest.skip("oracle/_ref not built (needs /root/reference at build time)")
    out = subprocess.check_output(["ldd", BIN], text=True)
    assert "libcudabulletproof_hip.so" in out


def test_reference_driver_crash_cause_on_cpu():
    """The CPU twin under AddressSanitizer + UBSan: no UBSan finding anywhere in the run, every line
    printed as by the plain CPU twin, and the one fault is the free of the uninitialised
    ip_proof at complete_bulletproof_test.cu:305 (field_vector_free <- inner_product_proof_free)."""
    if not (os.path.exists(ASAN) and os.path.exists(CPU)):
        pytest.skip("oracle/_ref not built (needs /root/reference at build time)")
    want, _ = _cpu_twin_lines()
    p = _run(ASAN, {"ASAN_OPTIONS": "detect_leaks=0", "UBSAN_OPTIONS": "print_stacktrace=1"})
    assert p.returncode != 0
    assert "runtime error" not in p.stderr, p.stderr[:4000]
    err = p.stderr
    assert "ERROR: AddressSanitizer" in err, err[-3000:]
    assert "0xaaaaaaaaaaaaaaaa" in err
    frames = [l for l in err.splitlines() if re.match(r"\s*#\d+ ", l)]
    ours = [l for l in frames if "/root/reference/" in l or "complete_bulletproof_test" in l]
    assert "field_vector_free" in ours[0] and "bulletproof_vectors.cu:29" in ours[0], ours
    assert "inner_product_proof_free" in ours[1], ours
    assert "main" in ours[2] and "complete_bulletproof_test.cu:305" in ours[2], ours
    got = _norm(p.stdout.splitlines())
    assert got == want
    assert got[-1].startswith(LAST_LINE)


@pytest.mark.gpu
def test_reference_driver_runs_on_our_library():
    """The drop-in binary on the GPU: the same lines as the CPU twin (less the reference's
    cuda_range_proof_verify-internal debug lines), both verifies SUCCESS, the out-of-range proof
    rejected, and then exactly the driver's own fault — SIGSEGV after the last line — as on the CPU."""
    if not (os.path.exists(BIN) and os.path.exists(CPU)):
        pytest.skip("oracle/_ref not built")
    want, cpu_err = _cpu_twin_lines()
    p = _run(BIN)
    got = _norm(p.stdout.splitlines())
    # complete_bulletproof_test.cu:179-191 / :247-255
    assert "CUDA Verification result: SUCCESS" in got, p.stdout[-3000:]
    assert "CPU Verification result: SUCCESS" in got
    assert any("FAILED (CORRECT)" in l for l in got)
    assert got[-1].startswith(LAST_LINE), got[-5:]
    assert got == _without_crv(want), "\n".join(l for l in got if l not in want)[:3000]
    # the refused proof's garbage ip_proof.n fails the length check (crv:140-143), on stderr, once
    assert p.stderr.count("Vector lengths must match for inner product verification") == 1, p.stderr[-2000:]
    assert "HIP error" not in p.stderr
    assert p.returncode == -signal.SIGSEGV, (p.returncode, p.stderr[-2000:])


def test_dropin_latency_harness_builds():
    """tests/dropin_latency.c compiles against include/cudabulletproof_hip.h and links the library."""
    import sys
    sys.path.insert(0, ROOT)
    import bench
    exe = bench.build_dropin_latency()
    assert "libcudabulletproof_hip.so" in subprocess.check_output(["ldd", exe], text=True)


@pytest.mark.gpu
def test_dropin_latency_wall_clock():
    """The drop-in cuda_range_proof_verify, one reference proof per call, timed by wall clock in a
    fresh process (tests/dropin_latency.c): every call returns the reference's verdict; the first
    call (engine set-up included, the HIP runtime's own start-up timed apart) and the warm calls
    are reported (bench.py configs0.dropin_latency carries the same figures)."""
    import sys
    sys.path.insert(0, ROOT)
    import bench
    r = bench.dropin_latency(ns=(16,), warm=10)["n16"]
    assert r["same_verdict_every_call"] and r["matches_reference_verdict"], r
    assert r["devices"] >= 1 and 0 < r["warm_median_ms"] < 1000 and r["first_call_ms"] < 10000, r
    print(r)
