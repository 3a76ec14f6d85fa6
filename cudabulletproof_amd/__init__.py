"""cudabulletproof_amd — MI355X (gfx950) engine for the MSM / inner-product-argument hot path
of ronantakizawa/cudabulletproof.

The compute path is libcudabulletproof_hip.so (hand-written HIP in csrc/, C ABI in
include/cudabulletproof_hip.h).  This module is a thin ctypes layer over that ABI:

* reference-named entry points (``cuda_point_vector_multi_scalar_mul``,
  ``cuda_range_proof_verify`` ...) that take numpy arrays in the reference's layouts
  and behave like the reference's C functions (cuda_bulletproof.h:13-84);
* a batched, device-resident verify (``RangeProofBatch`` + ``batch_range_proof_verify``)
  on torch CUDA tensors, used by bench.py.

There is no CPU fallback: if the library is missing or no GPU is present the calls
raise.  Layouts (numpy uint64): fe25519 (..., 4), ge25519 (..., 16) = X|Y|Z|T.
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
LIB_PATH = os.path.join(HERE, "libcudabulletproof_hip.so")
CSRC = os.path.join(HERE, "csrc")
SOURCES = ["bp_terms1.hip", "bp_terms2.hip", "bp_terms4.hip", "bp_terms16.hip", "bp_kernels.hip", "bp_prove.hip",
           "bp_pippenger.hip", "bp_capi.hip"]

_lib = None


class BulletproofError(RuntimeError):
    pass


def build(force=False, verbose=False):
    """Compile the HIP sources for gfx950 into LIB_PATH (in-tree, travels with the repo)."""
    srcs = [os.path.join(CSRC, s) for s in SOURCES]
    deps = srcs + [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".h")]
    deps.append(os.path.join(ROOT, "include", "cudabulletproof_hip.h"))
    if not force and os.path.exists(LIB_PATH):
        t = os.path.getmtime(LIB_PATH)
        if all(os.path.getmtime(d) <= t for d in deps):
            return LIB_PATH
    import tempfile
    flags = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-Wno-unused-result"]
    flags += os.environ.get("HIPBP_EXTRA_CFLAGS", "").split()   # A/B builds (e.g. -DBP_TERMS_OCC=3)
    with tempfile.TemporaryDirectory() as tmp:   # one hipcc per source, in parallel, then link
        objs = [os.path.join(tmp, os.path.basename(s) + ".o") for s in srcs]
        procs = []
        for s, o in zip(srcs, objs):
            cmd = ["hipcc"] + flags + ["-c", s, "-o", o]
            if verbose:
                print(" ".join(cmd))
            procs.append((cmd, subprocess.Popen(cmd)))
        for cmd, p in procs:
            if p.wait() != 0:
                raise subprocess.CalledProcessError(p.returncode, cmd)
        cmd = ["hipcc", "--offload-arch=gfx950", "-shared", "-fPIC", "-o", LIB_PATH + ".tmp"] + objs
        if verbose:
            print(" ".join(cmd))
        subprocess.check_call(cmd)
    os.replace(LIB_PATH + ".tmp", LIB_PATH)
    return LIB_PATH


_c = ctypes.c_void_p
_sz = ctypes.c_size_t


class FieldVector(ctypes.Structure):
    _fields_ = [("elements", _c), ("length", _sz)]


PointVector = FieldVector


class InnerProductProof(ctypes.Structure):   # bulletproof_vectors.h:65-74 (144 bytes)
    _fields_ = [("n", _sz), ("a", FieldVector), ("b", FieldVector), ("c", ctypes.c_uint64 * 4),
                ("L", PointVector), ("R", PointVector), ("L_len", _sz), ("x", ctypes.c_uint64 * 4)]


class RangeProofC(ctypes.Structure):   # bulletproof_range_proof.h:7-18 (880 bytes)
    _fields_ = [("V", ctypes.c_uint64 * 16), ("A", ctypes.c_uint64 * 16), ("S", ctypes.c_uint64 * 16),
                ("T1", ctypes.c_uint64 * 16), ("T2", ctypes.c_uint64 * 16), ("taux", ctypes.c_uint64 * 4),
                ("mu", ctypes.c_uint64 * 4), ("t", ctypes.c_uint64 * 4), ("ip_proof", InnerProductProof)]


class ProofBatchC(ctypes.Structure):   # hipbp_proof_batch
    _fields_ = [("count", _sz), ("n", _sz), ("ab_len", _sz), ("L_len", _sz)] + \
               [(k, _c) for k in ("V", "A", "S", "T1", "T2", "t", "a", "b", "c", "x", "L", "R", "taux", "mu", "Vp")]


class ProveInputC(ctypes.Structure):   # hipbp_prove_input
    _fields_ = [("count", _sz), ("n", _sz)] + [(k, _c) for k in ("v", "gamma", "sL", "sR", "rnd")]


class ProofOutC(ctypes.Structure):   # hipbp_proof_out
    _fields_ = [(k, _c) for k in ("V", "A", "S", "T1", "T2", "taux", "mu", "t", "c", "x", "a", "b", "L", "R", "valid")]


assert ctypes.sizeof(InnerProductProof) == 144 and ctypes.sizeof(RangeProofC) == 880

EXPORTS = [
    "cuda_point_vector_multi_scalar_mul", "cuda_point_vector_multi_scalar_mul_shared",
    "cuda_field_vector_inner_product", "cuda_field_vector_inner_product_shared",
    "cuda_batch_field_vector_inner_product", "cuda_batch_field_add", "cuda_batch_field_sub",
    "cuda_batch_field_mul", "cuda_batch_field_mul_karatsuba", "cuda_batch_field_square",
    "cuda_batch_field_invert", "cuda_soa_field_add", "cuda_range_proof_verify", "cuda_inner_product_verify",
    "cuda_benchmark_multi_scalar_mul", "cuda_benchmark_inner_product", "cuda_benchmark_field_operations",
    "cuda_benchmark_range_proof", "hipbp_last_error", "hipbp_device_count", "hipbp_batch_range_proof_verify",
    "hipbp_batch_range_proof_verify_std", "hipbp_batch_range_proof_verify_gens", "hipbp_batch_inner_product_verify", "hipbp_batch_generate_range_proof", "hipbp_msm",
    "hipbp_msm_pippenger", "hipbp_msm_pippenger_batch", "hipbp_msm_pippenger_windows",
    "hipbp_msm_pippenger_horner", "hipbp_msm_batch", "hipbp_msm_batch_gens", "hipbp_point_tree", "hipbp_field_op",
    "hipbp_sha_probe", "hipbp_sync", "hipbp_timing_enable",
    "hipbp_timing_collect", "hipbp_kernel_count", "hipbp_kernel_name", "hipbp_pipeline_create",
    "hipbp_pipeline_push", "hipbp_pipeline_flush", "hipbp_pipeline_depth", "hipbp_pipeline_destroy",
    "hipbp_pipeline_defer_msm",
    "hipbp_release_stream_workspaces",
]


def lib():
    """Load the HIP library (raises if it has not been built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise BulletproofError(f"{LIB_PATH} missing: run cudabulletproof_amd.build() (hipcc, gfx950)")
        # One HIP runtime per process: torch bundles its own libamdhip64.so.7 (same SONAME as
        # /opt/rocm's).  Importing torch first makes the dynamic loader bind this library to the
        # runtime torch uses, so device pointers, streams and torch.distributed interoperate.
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        L = ctypes.CDLL(LIB_PATH)
        L.hipbp_last_error.restype = ctypes.c_char_p
        for f in ("cuda_range_proof_verify", "cuda_inner_product_verify"):
            getattr(L, f).restype = ctypes.c_bool
        for f in ("hipbp_batch_range_proof_verify", "hipbp_batch_range_proof_verify_host",
                  "hipbp_batch_range_proof_verify_std", "hipbp_batch_range_proof_verify_gens",
                  "hipbp_batch_inner_product_verify", "hipbp_batch_generate_range_proof", "hipbp_msm",
                  "hipbp_msm_pippenger", "hipbp_msm_pippenger_batch", "hipbp_msm_pippenger_windows",
                  "hipbp_msm_pippenger_horner", "hipbp_msm_batch", "hipbp_msm_batch_gens", "hipbp_point_tree",
                  "hipbp_field_op", "hipbp_sha_probe", "hipbp_sync", "hipbp_device_count",
                  "hipbp_release_stream_workspaces"):
            getattr(L, f).restype = ctypes.c_int
        _lib = L
    return _lib


def require_gpu():
    n = lib().hipbp_device_count()
    if n < 1:
        raise BulletproofError("no HIP device visible: the engine has no CPU fallback")
    return n


def _chk(rc):
    if rc != 0:
        raise BulletproofError(lib().hipbp_last_error().decode())


def _p(a):
    return ctypes.c_void_p(a.ctypes.data)


def _u64(a, last):
    a = np.ascontiguousarray(a, dtype=np.uint64)
    if a.shape[-1] != last:
        raise ValueError(f"expected trailing dimension {last}, got {a.shape}")
    return a


# ====================================================================== reference-named host API
def cuda_point_vector_multi_scalar_mul(scalars, points, shared=False):
    """cuda_bulletproof.h:13 (shared: :17, cuda_point_vector_multi_scalar_mul_shared) — canonical-tree
    MSM of device-normalized terms; both entry points compute the same tree."""
    require_gpu()
    s, P = _u64(scalars, 4), _u64(points, 16)
    if len(s) != len(P):
        raise ValueError("Vector lengths must match for multi-scalar multiplication")
    out = np.zeros(16, np.uint64)
    sv, pv = FieldVector(_p(s).value, len(s)), PointVector(_p(P).value, len(P))
    f = lib().cuda_point_vector_multi_scalar_mul_shared if shared else lib().cuda_point_vector_multi_scalar_mul
    f(_p(out), ctypes.byref(sv), ctypes.byref(pv))
    return out


def cuda_field_vector_inner_product(a, b, shared=False):
    """cuda_bulletproof.h:22/:26 — the reference's GPU reduction order."""
    require_gpu()
    a, b = _u64(a, 4), _u64(b, 4)
    out = np.zeros(4, np.uint64)
    av, bv = FieldVector(_p(a).value, len(a)), FieldVector(_p(b).value, len(b))
    f = lib().cuda_field_vector_inner_product_shared if shared else lib().cuda_field_vector_inner_product
    f(_p(out), ctypes.byref(av), ctypes.byref(bv))
    return out


def cuda_batch_field_vector_inner_product(a_vectors, b_vectors):
    require_gpu()
    a, b = _u64(a_vectors, 4), _u64(b_vectors, 4)
    nv, n = a.shape[0], a.shape[1]
    av = (FieldVector * nv)(*[FieldVector(_p(a).value + i * n * 32, n) for i in range(nv)])
    bv = (FieldVector * nv)(*[FieldVector(_p(b).value + i * n * 32, n) for i in range(nv)])
    out = np.zeros((nv, 4), np.uint64)
    lib().cuda_batch_field_vector_inner_product(_p(out), av, bv, _sz(nv))
    return out


def _field(name, a, b=None):
    require_gpu()
    a = _u64(a, 4).reshape(-1, 4)
    out = np.zeros_like(a)
    if b is None:
        getattr(lib(), name)(_p(out), _p(a), _sz(len(a)))
    else:
        b = _u64(b, 4).reshape(-1, 4)
        if len(b) != len(a):
            raise ValueError("length mismatch")
        getattr(lib(), name)(_p(out), _p(a), _p(b), _sz(len(a)))
    return out


def cuda_batch_field_add(a, b):
    return _field("cuda_batch_field_add", a, b)


def cuda_batch_field_sub(a, b):
    return _field("cuda_batch_field_sub", a, b)


def cuda_batch_field_mul(a, b):
    return _field("cuda_batch_field_mul", a, b)


def cuda_batch_field_mul_karatsuba(a, b):
    return _field("cuda_batch_field_mul_karatsuba", a, b)


def cuda_batch_field_square(a):
    return _field("cuda_batch_field_square", a)


def cuda_batch_field_invert(a):
    return _field("cuda_batch_field_invert", a)


def cuda_soa_field_add(a, b):
    return _field("cuda_soa_field_add", a, b)


def _range_proof_struct(proof, n, keep):
    """proof: dict(head (100,) u64 = V,A,S,T1,T2 | taux,mu,t,c,x ; a, b (k,4); L, R (m,16))."""
    head = np.asarray(proof["head"], np.uint64)
    a, b = _u64(proof["a"], 4), _u64(proof["b"], 4)
    L, R = _u64(proof["L"], 16).reshape(-1, 16), _u64(proof["R"], 16).reshape(-1, 16)
    keep += [a, b, L, R]
    rp = RangeProofC()
    for i, k in enumerate(("V", "A", "S", "T1", "T2")):
        getattr(rp, k)[:] = [int(v) for v in head[16 * i:16 * i + 16]]
    for i, k in enumerate(("taux", "mu", "t")):
        getattr(rp, k)[:] = [int(v) for v in head[80 + 4 * i:84 + 4 * i]]
    ip = rp.ip_proof
    ip.n = n
    ip.a = FieldVector(_p(a).value, len(a))
    ip.b = FieldVector(_p(b).value, len(b))
    ip.c[:] = [int(v) for v in head[92:96]]
    ip.L = PointVector(_p(L).value, len(L))
    ip.R = PointVector(_p(R).value, len(R))
    ip.L_len = len(L)
    ip.x[:] = [int(v) for v in head[96:100]]
    return rp


def cuda_range_proof_verify(proof, V, n, G, H, g, h):
    """cuda_bulletproof.h:61 — one proof, host arrays, returns bool (crv:82 semantics)."""
    require_gpu()
    keep = []
    rp = _range_proof_struct(proof, n, keep)
    V, g, h = _u64(V, 16), _u64(g, 16), _u64(h, 16)
    G, H = _u64(G, 16), _u64(H, 16)
    gv, hv = PointVector(_p(G).value, len(G)), PointVector(_p(H).value, len(H))
    return bool(lib().cuda_range_proof_verify(ctypes.byref(rp), _p(V), _sz(n), ctypes.byref(gv), ctypes.byref(hv),
                                              _p(g), _p(h)))


def batch_range_proof_verify_host(proofs, V, n, G, H, g, h, num_gpus=0):
    """hipbp_batch_range_proof_verify_host: cuda_range_proof_verify over a list of proofs (the
    dicts cuda_range_proof_verify takes) packed as an array of the reference's RangeProof structs,
    sharded over num_gpus devices (0: all) from the current device on.  Host arrays in, (count,) bool
    verdicts out."""
    require_gpu()
    keep = []
    count = len(proofs)
    arr = (RangeProofC * max(count, 1))()
    for i, pr in enumerate(proofs):
        arr[i] = _range_proof_struct(pr, n, keep)
    V = _u64(V, 16).reshape(-1, 16)
    g, h = _u64(g, 16), _u64(h, 16)
    G, H = _u64(G, 16), _u64(H, 16)
    gv, hv = PointVector(_p(G).value, len(G)), PointVector(_p(H).value, len(H))
    ok = np.zeros(max(count, 1), np.uint8)
    _chk(lib().hipbp_batch_range_proof_verify_host(arr, _p(V), _sz(count), _sz(n), ctypes.byref(gv), ctypes.byref(hv),
                                                   _p(g), _p(h), ctypes.c_int(num_gpus), _p(ok)))
    return ok[:count].astype(bool)


def cuda_inner_product_verify(proof, P, G, H, Q):
    """cuda_bulletproof.h:72 — the IPA check alone (crv:130 semantics)."""
    require_gpu()
    keep = []
    G, H = _u64(G, 16), _u64(H, 16)
    rp = _range_proof_struct(proof, len(G), keep)
    P, Q = _u64(P, 16), _u64(Q, 16)
    gv, hv = PointVector(_p(G).value, len(G)), PointVector(_p(H).value, len(H))
    return bool(lib().cuda_inner_product_verify(ctypes.byref(rp.ip_proof), _p(P), ctypes.byref(gv), ctypes.byref(hv),
                                                _p(Q)))


# ====================================================================== batched device API (torch)
class RangeProofBatch:
    """A batch of proofs in the flat wire format, resident on a torch CUDA device.

    Tensors are int64 views of the u64 limbs: V/A/S/T1/T2 (B,16), t/c/x (B,4),
    a/b (B,ab_len,4), L/R (B,L_len,16).  Optional (range_proof_verify semantics only):
    taux/mu (B,4) and Vp (B,16), the proof's own V (default: V).
    """

    FIELDS = ("V", "A", "S", "T1", "T2", "t", "a", "b", "c", "x", "L", "R")
    OPTIONAL = ("taux", "mu", "Vp")

    def __init__(self, n, **tensors):
        self.n = int(n)
        for k in self.FIELDS:
            setattr(self, k, tensors[k].contiguous())
        for k in self.OPTIONAL:
            v = tensors.get(k)
            setattr(self, k, v.contiguous() if v is not None else None)
        self.count = int(self.V.shape[0])
        self.ab_len = int(self.a.shape[1])
        self.L_len = int(self.L.shape[1])

    @classmethod
    def from_numpy(cls, n, arrays, device):
        import torch
        t = {k: torch.from_numpy(np.ascontiguousarray(arrays[k]).view(np.int64)).to(device)
             for k in cls.FIELDS + cls.OPTIONAL if arrays.get(k) is not None}
        return cls(n, **t)

    def c_struct(self):
        s = ProofBatchC(self.count, self.n, self.ab_len, self.L_len)
        for k in self.FIELDS:
            setattr(s, k, getattr(self, k).data_ptr())
        for k in self.OPTIONAL:
            v = getattr(self, k)
            setattr(s, k, v.data_ptr() if v is not None else None)
        return s

    def nbytes(self):
        return sum(getattr(self, k).numel() * 8 for k in self.FIELDS)


def _stream_ptr(stream):
    if stream is None:
        import torch
        stream = torch.cuda.current_stream()
    return ctypes.c_void_p(stream.cuda_stream)


def batch_range_proof_verify(batch, G, H, g, h, ok, P_out=None, check_out=None, stream=None):
    """Enqueue cuda_range_proof_verify over the whole batch on `stream` (asynchronous).

    G/H: (n,16) int64 CUDA tensors, g/h: (16,), ok: (B,) uint8, P_out/check_out: (B,16) or None.
    """
    s = batch.c_struct()
    _chk(lib().hipbp_batch_range_proof_verify(
        ctypes.byref(s), _c(G.data_ptr()), _c(H.data_ptr()), _c(g.data_ptr()), _c(h.data_ptr()), _c(ok.data_ptr()),
        _c(P_out.data_ptr()) if P_out is not None else None,
        _c(check_out.data_ptr()) if check_out is not None else None, _stream_ptr(stream)))


def batch_range_proof_verify_gens(batch, gens, ok, P_out=None, check_out=None, stream=None):
    """batch_range_proof_verify with a Generators set's generators and prefix tables
    (hipbp_batch_range_proof_verify_gens): same bits, the table-started scalar multiplications."""
    s = batch.c_struct()
    _chk(lib().hipbp_batch_range_proof_verify_gens(
        ctypes.byref(s), _c(gens.h), _c(ok.data_ptr()), _c(P_out.data_ptr()) if P_out is not None else None,
        _c(check_out.data_ptr()) if check_out is not None else None, _stream_ptr(stream)))


def batch_range_proof_verify_std(batch, G, H, g, h, ok, P_out=None, check_out=None, flags_out=None, poly_out=None,
                                 stream=None):
    """Enqueue range_proof_verify semantics (bulletproof_range_proof.cu:1717) over the
    batch (needs batch.taux/mu).  flags_out (B,) uint8: bit0 V match, bit1 range check, bit2
    polynomial identity methods 1|2, bit3 method 3, bit4 method 4, bit5 inner_product_verify;
    poly_out (B,4,16): left, right, chal*left, chal*right."""
    s = batch.c_struct()
    opt = lambda t: _c(t.data_ptr()) if t is not None else None
    _chk(lib().hipbp_batch_range_proof_verify_std(
        ctypes.byref(s), _c(G.data_ptr()), _c(H.data_ptr()), _c(g.data_ptr()), _c(h.data_ptr()), _c(ok.data_ptr()),
        opt(P_out), opt(check_out), opt(flags_out), opt(poly_out), _stream_ptr(stream)))


def batch_inner_product_verify(batch, P, G, H, Q, ok, check_out=None, stream=None):
    s = batch.c_struct()
    _chk(lib().hipbp_batch_inner_product_verify(
        ctypes.byref(s), _c(P.data_ptr()), _c(G.data_ptr()), _c(H.data_ptr()), _c(Q.data_ptr()), _c(ok.data_ptr()),
        _c(check_out.data_ptr()) if check_out is not None else None, _stream_ptr(stream)))


class Generators:
    """hipbp_gens_create: a device snapshot of the generators G (n,16), H (n,16), g, h (16,) and,
    with prefix_bits > 0, their fixed-base prefix tables ((2n + 2) * 2^bits * 128 bytes).  Pass it
    to batch_generate_range_proof(gens=...) and VerifyPipeline.use_gens(); results keep their bits."""

    def __init__(self, n, G, H, g, h, prefix_bits=0, stream=None):
        L = lib()
        L.hipbp_gens_create.restype = ctypes.c_void_p
        self.n, self.bits = int(n), int(prefix_bits)
        self.h = L.hipbp_gens_create(_sz(n), _c(G.data_ptr()), _c(H.data_ptr()), _c(g.data_ptr()), _c(h.data_ptr()),
                                     ctypes.c_int(self.bits), _stream_ptr(stream))
        if not self.h:
            raise BulletproofError(L.hipbp_last_error().decode())

    def nbytes_tables(self):
        return (2 * self.n + 2) * (1 << self.bits) * 128 if self.bits else 0

    def close(self):
        if self.h:
            lib().hipbp_gens_destroy(_c(self.h))
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def batch_generate_range_proof(n, v, gamma, sL, sR, rnd, G, H, g, h, stream=None, gens=None):
    """generate_range_proof (bulletproof_range_proof.cu:1159) over a batch, on the GPU.

    v, gamma (B,4); sL, sR (B,n,4); rnd (B,4,4) = alpha, rho, tau1, tau2: int64 CUDA tensors of the
    u64 limbs (the random scalars exactly as generate_random_scalar produced them).  Returns a dict
    of CUDA tensors in RangeProofBatch layout (V, A, S, T1, T2, t, a, b, c, x, L, R, taux, mu) plus
    "valid" (B,) uint8; RangeProofBatch(n, **out) verifies it directly."""
    import contextlib

    import torch
    B = int(v.shape[0])
    Lr = int(n).bit_length() - 1
    dev = v.device
    # every output element is written by the prover (refused proofs get the reference's zeroed
    # proof), so the buffers are allocated uninitialised on the stream the prover runs on
    with torch.cuda.stream(stream) if stream is not None else contextlib.nullcontext():
        z = lambda *shape: torch.empty(*shape, dtype=torch.int64, device=dev)
        out = dict(V=z(B, 16), A=z(B, 16), S=z(B, 16), T1=z(B, 16), T2=z(B, 16), taux=z(B, 4), mu=z(B, 4),
                   t=z(B, 4), c=z(B, 4), x=z(B, 4), a=z(B, 1, 4), b=z(B, 1, 4), L=z(B, max(Lr, 0), 16),
                   R=z(B, max(Lr, 0), 16), valid=torch.empty(B, dtype=torch.uint8, device=dev))
    ins = [t.contiguous() for t in (v, gamma, sL, sR, rnd)]
    ic = ProveInputC(B, int(n), *[t.data_ptr() for t in ins])
    oc = ProofOutC(*[out[k].data_ptr() if out[k].numel() else None for k in
                     ("V", "A", "S", "T1", "T2", "taux", "mu", "t", "c", "x", "a", "b", "L", "R", "valid")])
    if gens is not None:   # the set's generators and prefix tables (G, H, g, h are not read)
        _chk(lib().hipbp_batch_generate_range_proof_gens(ctypes.byref(ic), _c(gens.h), ctypes.byref(oc),
                                                         _stream_ptr(stream)))
    else:
        _chk(lib().hipbp_batch_generate_range_proof(ctypes.byref(ic), _c(G.data_ptr()), _c(H.data_ptr()),
                                                    _c(g.data_ptr()), _c(h.data_ptr()), ctypes.byref(oc),
                                                    _stream_ptr(stream)))
    out["_keep"] = ins
    return out


def msm(result, scalars, points, stream=None):
    """Canonical-tree MSM on CUDA tensors: result (16,), scalars (n,4), points (n,16)."""
    _chk(lib().hipbp_msm(_c(result.data_ptr()), _c(scalars.data_ptr()), _c(points.data_ptr()),
                         _sz(points.shape[0]), _stream_ptr(stream)))


def msm_batch(results, scalars, points, stream=None):
    """count canonical-tree MSMs over the same points: results (count,16), scalars (count*n,4) or
    (count,n,4), points (n,16); CUDA tensors."""
    n = points.shape[0]
    count = results.shape[0]
    if scalars.numel() != count * n * 4:
        raise BulletproofError("msm_batch: scalars must hold count * n rows")
    _chk(lib().hipbp_msm_batch(_c(results.data_ptr()), _c(scalars.data_ptr()), _c(points.data_ptr()), _sz(n),
                               _sz(count), _stream_ptr(stream)))


def msm_batch_gens(results, scalars, gens, stream=None):
    """msm_batch over a Generators set's G||H (2n points) with its prefix tables: results (count,16),
    scalars (count*2n,4); the same bits as msm_batch(results, scalars, cat(G, H))."""
    count, n2 = results.shape[0], 2 * gens.n
    if scalars.numel() != count * n2 * 4:
        raise BulletproofError("msm_batch_gens: scalars must hold count * 2n rows")
    _chk(lib().hipbp_msm_batch_gens(_c(results.data_ptr()), _c(scalars.data_ptr()), _c(gens.h), _sz(count),
                                    _stream_ptr(stream)))


def msm_pippenger(result, scalars, points, window_bits=12, stream=None):
    """Pippenger bucket MSM on CUDA tensors (labelled alternative: not the reference's MSM bits,
    see include/cudabulletproof_hip.h)."""
    _chk(lib().hipbp_msm_pippenger(_c(result.data_ptr()), _c(scalars.data_ptr()), _c(points.data_ptr()),
                                   _sz(points.shape[0]), ctypes.c_int(window_bits), _stream_ptr(stream)))


def msm_pippenger_batch(results, scalars, points, window_bits=12, stream=None):
    """count Pippenger MSMs over the same points: results (count,16), scalars (count*n,4) or
    (count,n,4), points (n,16), device tensors."""
    count, n = results.shape[0], points.shape[0]
    if scalars.numel() != count * n * 4:
        raise BulletproofError("msm_pippenger_batch: scalars must hold count * n rows")
    _chk(lib().hipbp_msm_pippenger_batch(_c(results.data_ptr()), _c(scalars.data_ptr()), _c(points.data_ptr()),
                                         _sz(n), _sz(count), ctypes.c_int(window_bits), _stream_ptr(stream)))


def pippenger_num_windows(window_bits=12):
    return (256 + int(window_bits) - 1) // int(window_bits)


def msm_pippenger_windows(window_sums, scalars, points, w_begin, w_end, window_bits=12, stream=None):
    """Window sums S_w, w in [w_begin, w_end), of the Pippenger MSM into window_sums[w] (a (W,16)
    device tensor, W = pippenger_num_windows; other rows untouched)."""
    W = pippenger_num_windows(window_bits)
    if window_sums.numel() != W * 16:
        raise BulletproofError(f"msm_pippenger_windows: window_sums must be ({W}, 16)")
    if scalars.numel() != points.shape[0] * 4:
        raise BulletproofError("msm_pippenger_windows: one scalar per point")
    _chk(lib().hipbp_msm_pippenger_windows(_c(window_sums.data_ptr()), _c(scalars.data_ptr()),
                                           _c(points.data_ptr()), _sz(points.shape[0]), ctypes.c_int(window_bits),
                                           ctypes.c_int(w_begin), ctypes.c_int(w_end), _stream_ptr(stream)))


def msm_pippenger_horner(results, window_sums, window_bits=12, stream=None):
    """Horner over all W window sums: results (count,16) or (16,), window_sums (count*W,16)."""
    W = pippenger_num_windows(window_bits)
    count = results.numel() // 16
    if window_sums.numel() != count * W * 16:
        raise BulletproofError(f"msm_pippenger_horner: window_sums must hold count * {W} rows")
    _chk(lib().hipbp_msm_pippenger_horner(_c(results.data_ptr()), _c(window_sums.data_ptr()), _sz(count),
                                          ctypes.c_int(window_bits), _stream_ptr(stream)))


def release_stream_workspaces(stream=None):
    """hipbp_release_stream_workspaces: free every workspace cached for `stream` on the current
    device (MSM, prover, one-shot pipelines, Pippenger pair); call before dropping a stream."""
    _chk(lib().hipbp_release_stream_workspaces(_stream_ptr(stream)))


def point_tree(result, points, stream=None):
    """Canonical tree over device points (the MSM's reduction half): result (16,), points (n,16)."""
    _chk(lib().hipbp_point_tree(_c(result.data_ptr()), _c(points.data_ptr()), _sz(points.shape[0]),
                                _stream_ptr(stream)))


def field_op(op, r, a, b=None, stream=None):
    ops = {"add": 0, "sub": 1, "mul": 2, "square": 3, "soa_add": 4, "invert": 5, "fold": 6, "sq": 7,
           "addsub_add": 8, "addsub_sub": 9,   # 8/9: the fused add/sub block's sum / difference
           "mul_q4": 10,   # 10: fe25519_mul as the drain forms' quad-split product (fe_mul_q4)
           "mul_k": 11,    # 11: fe25519_mul(a, k), the point operations' product by the constant (fe_mul_k)
           "mul_q4_k": 12,   # 12: the same split over a lane quad (fe_mul_q4_k, the drain forms' C)
           # the row step's latency forms (13, 15/16, 19) and deferred rare-edge forms (14, 17/18, 20)
           "add_lat": 13, "add_defer": 14, "addsub_lat_add": 15, "addsub_lat_sub": 16,
           "addsub_defer_add": 17, "addsub_defer_sub": 18, "fold_lat": 19, "fold_defer": 20}
    _chk(lib().hipbp_field_op(ops[op], _c(r.data_ptr()), _c(a.data_ptr()), _c(b.data_ptr()) if b is not None else None,
                              _sz(a.shape[0]), _stream_ptr(stream)))


def sha_probe(kind, out, inp, stream=None):
    """hipbp_sha_probe: the verify path's SHA-256 message shapes on the device (kind 0 y, 1 z, 2 x,
    3 inner-product round, 4 prover IPA start, 5 raw digest of four values); inp (N, 6, 4), out (N, 4)."""
    _chk(lib().hipbp_sha_probe(int(kind), _c(out.data_ptr()), _c(inp.data_ptr()), _sz(inp.shape[0]),
                               _stream_ptr(stream)))


# ====================================================================== per-kernel timing
def timing_enable(on=True):
    """Record HIP events around each verify-pipeline kernel launch (resets the totals)."""
    L = lib()
    L.hipbp_timing_enable.restype = ctypes.c_int
    _chk(L.hipbp_timing_enable(1 if on else 0))


def timing_collect():
    """{kernel_name: (total_ms, launches)} accumulated since timing_enable()."""
    L = lib()
    L.hipbp_kernel_name.restype = ctypes.c_char_p
    L.hipbp_timing_collect.restype = ctypes.c_int
    k = L.hipbp_kernel_count()
    ms = (ctypes.c_double * k)()
    cnt = (ctypes.c_uint64 * k)()
    _chk(L.hipbp_timing_collect(ms, cnt))
    return {L.hipbp_kernel_name(i).decode(): (ms[i], cnt[i]) for i in range(k)}


# ====================================================================== streaming verify pipeline
class VerifyPipeline:
    """hipbp_pipeline_*: up to `depth` batches in flight; each push runs one tick in which
    every in-flight batch advances one stage (stage 0 / fold round r / final).  A batch's
    outputs are complete after depth-1 further pushes or flush()."""

    def __init__(self, max_batch, n, G, H, h, range_mode=True, stream=None, g=None):
        """range_mode: True/1 cuda_range_proof_verify, 2 range_proof_verify (needs g), False/0
        cuda_inner_product_verify (h = Q)."""
        L = lib()
        L.hipbp_pipeline_create.restype = ctypes.c_void_p
        L.hipbp_pipeline_push.restype = ctypes.c_int
        L.hipbp_pipeline_flush.restype = ctypes.c_int
        L.hipbp_pipeline_depth.restype = ctypes.c_int
        self._keep = (G, H, h, g)
        self.stream = stream   # the torch stream the ticks run on (None: the null stream)
        self.mode = int(range_mode)
        self.h = L.hipbp_pipeline_create(_sz(max_batch), _sz(n), self.mode, _c(G.data_ptr()), _c(H.data_ptr()),
                                         _c(g.data_ptr()) if g is not None else None, _c(h.data_ptr()),
                                         _stream_ptr(stream))
        if not self.h:
            raise BulletproofError(L.hipbp_last_error().decode())
        self.depth = L.hipbp_pipeline_depth(_c(self.h))

    def push(self, batch, ok=None, P_out=None, check_out=None, P_in=None, flags_out=None, poly_out=None):
        s = batch.c_struct() if batch is not None else None
        opt = lambda t: _c(t.data_ptr()) if t is not None else None
        _chk(lib().hipbp_pipeline_push(
            _c(self.h), ctypes.byref(s) if s is not None else None, opt(P_in), opt(ok), opt(P_out), opt(check_out),
            opt(flags_out), opt(poly_out)))

    def flush(self):
        _chk(lib().hipbp_pipeline_flush(_c(self.h)))

    def use_gens(self, gens):
        """hipbp_pipeline_use_gens: generators and prefix tables from a Generators set."""
        _chk(lib().hipbp_pipeline_use_gens(_c(self.h), _c(gens.h)))
        self._gens = gens

    def defer_msm(self, on=True):
        """hipbp_pipeline_defer_msm: split stage 0 for the batches pushed from now on (the MSM
        terms, t*h and c*Q as RK_MSMT chunks inside the batch's fold-round ticks, stages 2 .. L, on
        the pipeline's own stream; the lane trees at the final-terms tick); same bits.  Raises
        BulletproofError where the split does not apply (inner-product mode, n above the lane-tree
        limit, n > 512)."""
        _chk(lib().hipbp_pipeline_defer_msm(_c(self.h), ctypes.c_int(1 if on else 0)))

    def prefix_tables(self, bits):
        """hipbp_pipeline_prefix_tables: fixed-base prefix tables of the generators (same bits,
        fewer point operations); bits = 0 frees them.  Synchronous; the pipeline must be idle."""
        _chk(lib().hipbp_pipeline_prefix_tables(_c(self.h), ctypes.c_int(int(bits))))

    def close(self):
        if self.h:
            lib().hipbp_pipeline_destroy(_c(self.h))
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
