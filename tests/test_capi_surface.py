"""CPU-side checks of the drop-in boundary: the HIP library builds for gfx950, loads, and
exports every entry point include/cudabulletproof_hip.h declares (no compute without a GPU);
the struct layouts match the reference's; the product never reaches into oracle/."""
import ctypes
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "cudabulletproof_hip.h")

# cuda_bulletproof.h:13-84 — every function the reference's header declares
REFERENCE_SURFACE = [
    "cuda_point_vector_multi_scalar_mul", "cuda_point_vector_multi_scalar_mul_shared",
    "cuda_field_vector_inner_product", "cuda_field_vector_inner_product_shared", "cuda_batch_field_add",
    "cuda_batch_field_sub", "cuda_batch_field_mul", "cuda_batch_field_square", "cuda_batch_field_invert",
    "cuda_soa_field_add", "cuda_range_proof_verify", "cuda_inner_product_verify", "cuda_benchmark_multi_scalar_mul",
    "cuda_benchmark_inner_product", "cuda_benchmark_field_operations", "cuda_benchmark_range_proof",
]


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:const\s+)?[A-Za-z_][\w\s\*]*?\b([a-z_][a-z0-9_]*)\s*\(", src, flags=re.M)))


@pytest.fixture(scope="module")
def libpath():
    import cudabulletproof_amd as m
    return m.build()


def test_header_declares_reference_surface():
    decl = declared_functions()
    for f in REFERENCE_SURFACE:
        assert f in decl, f


def test_library_exports_every_declared_symbol(libpath):
    out = subprocess.check_output(["nm", "-D", "--defined-only", libpath], text=True)
    exported = {line.split()[-1] for line in out.splitlines() if " T " in line}
    missing = [f for f in declared_functions() if f not in exported]
    assert not missing, missing


def test_library_loads_and_is_gfx950(libpath):
    import cudabulletproof_amd as m
    L = m.lib()
    for f in m.EXPORTS:
        assert hasattr(L, f), f
    # the embedded code object targets gfx950
    blob = open(libpath, "rb").read()
    assert b"gfx950" in blob


def test_struct_layouts():
    import cudabulletproof_amd as m
    assert ctypes.sizeof(m.InnerProductProof) == 144
    assert ctypes.sizeof(m.RangeProofC) == 880
    assert m.RangeProofC.ip_proof.offset == 736
    for name, off in (("n", 0), ("a", 8), ("b", 24), ("c", 40), ("L", 72), ("R", 88), ("L_len", 104), ("x", 112)):
        assert getattr(m.InnerProductProof, name).offset == off, name


def test_product_does_not_use_oracle():
    pkg = os.path.join(ROOT, "cudabulletproof_amd")
    for dp, _, files in os.walk(pkg):
        for f in files:
            if f.endswith((".py", ".hip", ".h", ".cpp")):
                txt = open(os.path.join(dp, f)).read()
                assert "oracle" not in txt.replace("no CPU fallback", ""), f


def test_no_device_means_no_result():
    """With no HIP device visible the engine has no CPU fallback: the Python mirror raises before
    touching the C ABI, and the C ABI itself (cuda_range_proof_verify, reference error behaviour:
    device error -> stderr + exit, cuda_bulletproof_kernels.cu:13-21) ends the process instead of
    returning a verdict.  Run in child processes with every device hidden."""
    import sys
    env = dict(os.environ, HIP_VISIBLE_DEVICES="-1", ROCR_VISIBLE_DEVICES="-1")
    py = ("import numpy as np, cudabulletproof_amd as bp\n"
          "d = np.load('tests/golden/proofs_n16.npz')\n"
          "try:\n"
          "    bp.cuda_range_proof_verify({}, d['V'][0], 16, d['G'], d['H'], d['g'], d['h'])\n"
          "    print('RESULT')\n"
          "except bp.BulletproofError as e:\n"
          "    print('RAISED', e)\n")
    r = subprocess.run([sys.executable, "-c", py], cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert "RAISED" in r.stdout and "no CPU fallback" in r.stdout and "RESULT" not in r.stdout, (r.stdout, r.stderr)
    # the C ABI called directly (bypassing the Python check) on the same well-formed proof: no verdict
    # comes back
    py2 = ("import ctypes, sys, numpy as np, cudabulletproof_amd as bp\n"
           "sys.path.insert(0, 'tests')\n"
           "from test_gpu_parity import _proof\n"
           "d = np.load('tests/golden/proofs_n16.npz')\n"
           "keep = []\n"
           "rp = bp._range_proof_struct(_proof(d, 0), 16, keep)\n"
           "u = lambda a: np.ascontiguousarray(a, np.uint64)\n"
           "V, g, h, G, H = u(d['V'][0]), u(d['g']), u(d['h']), u(d['G']), u(d['H'])\n"
           "p = lambda a: ctypes.c_void_p(a.ctypes.data)\n"
           "gv, hv = bp.PointVector(p(G).value, len(G)), bp.PointVector(p(H).value, len(H))\n"
           "ok = bp.lib().cuda_range_proof_verify(ctypes.byref(rp), p(V), ctypes.c_size_t(16), ctypes.byref(gv), "
           "ctypes.byref(hv), p(g), p(h))\n"
           "print('RESULT', ok)\n")
    r = subprocess.run([sys.executable, "-c", py2], cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode != 0 and "RESULT" not in r.stdout and "HIP error" in r.stderr, (r.returncode, r.stdout, r.stderr)
