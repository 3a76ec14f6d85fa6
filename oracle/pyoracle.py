"""pyoracle — TEST INFRASTRUCTURE ONLY.

ctypes bindings for the CPU restatement (oracle/libbp_oracle.so) and, when it
has been built, the reference build (oracle/_ref/libbpref.so).  Imported only by
tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg.

Array conventions (the reference's own layouts):
  fe25519 -> numpy uint64 (..., 4)   little-endian limbs   (curve25519_ops.h:15-17)
  ge25519 -> numpy uint64 (..., 16)  X|Y|Z|T limbs         (curve25519_ops.h:20-25)
  head    -> numpy uint64 (100,)     V,A,S,T1,T2 (5x16) then taux,mu,t,c,x (5x4)
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ORACLE_SO = os.path.join(HERE, "libbp_oracle.so")
REF_SO = os.path.join(HERE, "_ref", "libbpref.so")

HEAD_WORDS = 5 * 16 + 5 * 4
_c = ctypes.c_void_p
_sz = ctypes.c_size_t


def build():
    """Compile the C restatement (and the reference build when /root/reference exists)."""
    subprocess.check_call(["make", "-s", "-C", HERE, "libbp_oracle.so"])
    if os.path.isdir("/root/reference"):
        subprocess.check_call([os.path.join(HERE, "build_ref.sh")], stdout=subprocess.DEVNULL)


def _p(a):
    return a.ctypes.data_as(_c)


def fe(n=None):
    return np.zeros((4,) if n is None else (n, 4), np.uint64)


def ge(n=None):
    return np.zeros((16,) if n is None else (n, 16), np.uint64)


class _Lib:
    prefix = ""

    def __init__(self, path):
        self.lib = ctypes.CDLL(path)

    def f(self, name):
        return getattr(self.lib, self.prefix + name)


class Oracle(_Lib):
    """The C restatement (bp_oracle.c)."""

    prefix = "orc_"

    def __init__(self, path=ORACLE_SO):
        if not os.path.exists(path):
            build()
        super().__init__(path)
        self.lib.orc_cuda_range_proof_verify.restype = ctypes.c_int
        self.lib.orc_cuda_inner_product_verify.restype = ctypes.c_int
        self.lib.orc_range_proof_verify.restype = ctypes.c_int
        self.lib.orc_generate_range_proof.restype = ctypes.c_int

    # field ------------------------------------------------------------
    def _fe2(self, name, f, g):
        h = fe()
        self.f(name)(_p(h), _p(np.ascontiguousarray(f, np.uint64)), _p(np.ascontiguousarray(g, np.uint64)))
        return h

    def fe_add(self, f, g):
        return self._fe2("fe_add", f, g)

    def fe_sub(self, f, g):
        return self._fe2("fe_sub", f, g)

    def fe_mul(self, f, g):
        return self._fe2("fe_mul", f, g)

    def fe_invert(self, f):
        h = fe()
        self.f("fe_invert")(_p(h), _p(np.ascontiguousarray(f, np.uint64)))
        return h

    def fe_square_kernel(self, f):
        h = fe()
        self.f("fe_square_kernel")(_p(h), _p(np.ascontiguousarray(f, np.uint64)))
        return h

    def fe_tobytes(self, f):
        b = np.zeros(32, np.uint8)
        self.f("fe_tobytes")(_p(b), _p(np.ascontiguousarray(f, np.uint64)))
        return b

    # points -----------------------------------------------------------
    def ge_add(self, p, q):
        r = ge()
        self.f("ge_add")(_p(r), _p(np.ascontiguousarray(p, np.uint64)), _p(np.ascontiguousarray(q, np.uint64)))
        return r

    def ge_scalarmult(self, s32, p):
        r = ge()
        self.f("ge_scalarmult")(_p(r), _p(np.ascontiguousarray(s32, np.uint8)), _p(np.ascontiguousarray(p, np.uint64)))
        return r

    def ge_normalize_host(self, p):
        q = np.array(p, np.uint64)
        self.f("ge_normalize_host")(_p(q))
        return q

    def ge_normalize_dev(self, p):
        q = np.array(p, np.uint64)
        self.f("ge_normalize_dev")(_p(q))
        return q

    # vectors ----------------------------------------------------------
    def msm_canon(self, s, P):
        r = ge()
        s = np.ascontiguousarray(s, np.uint64)
        P = np.ascontiguousarray(P, np.uint64)
        self.f("msm_canon")(_p(r), _p(s), _p(P), _sz(len(P)))
        return r

    def point_tree(self, P):
        r = ge()
        P = np.ascontiguousarray(P, np.uint64).reshape(-1, 16)
        self.f("point_tree")(_p(r), _p(P), _sz(len(P)))
        return r

    def msm_pippenger(self, s, P, c=12):
        r = ge()
        s = np.ascontiguousarray(s, np.uint64)
        P = np.ascontiguousarray(P, np.uint64)
        self.f("msm_pippenger")(_p(r), _p(s), _p(P), _sz(len(P)), ctypes.c_int(c))
        return r

    def pippenger_windows(self, s, P, c, w0, w1):
        """Window sums S_w for w in [w0, w1) (rows 0 .. w1 - w0 - 1 of the result)."""
        W = (256 + c - 1) // c
        Sw = np.zeros((W, 16), np.uint64)
        s = np.ascontiguousarray(s, np.uint64)
        P = np.ascontiguousarray(P, np.uint64)
        self.f("pippenger_windows")(_p(Sw), _p(s), _p(P), _sz(len(P)), ctypes.c_int(c), ctypes.c_int(w0),
                                    ctypes.c_int(w1))
        return Sw[w0:w1].copy()

    def pippenger_horner(self, Sw, c):
        r = ge()
        Sw = np.ascontiguousarray(Sw, np.uint64).reshape(-1, 16)
        assert len(Sw) == (256 + c - 1) // c
        self.f("pippenger_horner")(_p(r), _p(Sw), ctypes.c_int(c))
        return r

    def msm_cpu(self, s, P):
        r = ge()
        s = np.ascontiguousarray(s, np.uint64)
        P = np.ascontiguousarray(P, np.uint64)
        self.f("msm_cpu")(_p(r), _p(s), _p(P), _sz(len(P)))
        return r

    def inner_product(self, a, b):
        r = fe()
        a = np.ascontiguousarray(a, np.uint64)
        b = np.ascontiguousarray(b, np.uint64)
        self.f("inner_product")(_p(r), _p(a), _p(b), _sz(len(a)))
        return r

    def ip_gpu(self, a, b, shared=False):
        r = fe()
        a = np.ascontiguousarray(a, np.uint64)
        b = np.ascontiguousarray(b, np.uint64)
        self.f("ip_gpu_shared" if shared else "ip_gpu")(_p(r), _p(a), _p(b), _sz(len(a)))
        return r

    def ip_gpu_batch(self, a, b):
        a = np.ascontiguousarray(a, np.uint64)
        b = np.ascontiguousarray(b, np.uint64)
        r = fe(a.shape[0])
        self.f("ip_gpu_batch")(_p(r), _p(a), _p(b), _sz(a.shape[1]), _sz(a.shape[0]))
        return r

    def base_points(self, n, seed_byte):
        out = ge(n)
        seed = np.zeros(32, np.uint8)
        seed[0] = seed_byte
        self.f("base_points")(_p(out), _sz(n), _p(seed))
        return out

    def gh(self):
        g, h = ge(), ge()
        self.f("gh")(_p(g), _p(h))
        return g, h

    def sha256(self, data):
        buf = np.frombuffer(bytes(data), np.uint8).copy()
        out = np.zeros(32, np.uint8)
        self.f("sha256")(_p(out), _p(buf) if len(buf) else None, _sz(len(buf)))
        return out.tobytes()

    # verify -----------------------------------------------------------
    def cuda_range_proof_verify(self, head, V, n, a, b, L, R, G, H, g, h, trace=False):
        """crv:82 semantics. Returns (ok, P, check_point, Gtrace, Htrace)."""
        head = np.ascontiguousarray(head, np.uint64)
        a = np.ascontiguousarray(a, np.uint64).reshape(-1, 4)
        b = np.ascontiguousarray(b, np.uint64).reshape(-1, 4)
        L = np.ascontiguousarray(L, np.uint64).reshape(-1, 16)
        R = np.ascontiguousarray(R, np.uint64).reshape(-1, 16)
        P, chk = ge(), ge()
        chk[:] = 0
        Gt = ge(max(n - 1, 1)) if trace else None
        Ht = ge(max(n - 1, 1)) if trace else None
        ok = self.f("cuda_range_proof_verify")(
            _p(head), _p(np.ascontiguousarray(V, np.uint64)), _sz(n), _p(a), _p(b), _sz(len(a)), _p(L), _p(R),
            _sz(len(L)), _p(np.ascontiguousarray(G, np.uint64)), _p(np.ascontiguousarray(H, np.uint64)),
            _p(np.ascontiguousarray(g, np.uint64)), _p(np.ascontiguousarray(h, np.uint64)), _p(P), _p(chk),
            _p(Gt) if trace else None, _p(Ht) if trace else None)
        return bool(ok), P, chk, Gt, Ht


    def cuda_inner_product_verify(self, n, a, b, c, L, R, x, P, G, H, Q, trace=False):
        """orc_cuda_inner_product_verify -> (ok, check_point, Gtrace, Htrace)."""
        a, b = np.ascontiguousarray(a, np.uint64).reshape(-1, 4), np.ascontiguousarray(b, np.uint64).reshape(-1, 4)
        L, R = np.ascontiguousarray(L, np.uint64).reshape(-1, 16), np.ascontiguousarray(R, np.uint64).reshape(-1, 16)
        chk = ge()
        Gt = ge(max(n - 1, 1)) if trace else None
        Ht = ge(max(n - 1, 1)) if trace else None
        ok = self.f("cuda_inner_product_verify")(
            _sz(n), _p(a), _p(b), _sz(len(a)), _p(np.ascontiguousarray(c, np.uint64)), _p(L), _p(R), _sz(len(L)),
            _p(np.ascontiguousarray(x, np.uint64)), _p(np.ascontiguousarray(P, np.uint64)),
            _p(np.ascontiguousarray(G, np.uint64)), _p(np.ascontiguousarray(H, np.uint64)),
            _p(np.ascontiguousarray(Q, np.uint64)), _p(chk), _p(Gt) if trace else None, _p(Ht) if trace else None)
        return bool(ok), chk, Gt, Ht


    RPV_KEYS = ("vmatch", "range_ok", "poly_ok", "poly_m1", "poly_m2", "poly_m3", "poly_m4", "ip_ok")
    RPV_PTS = ("left", "right", "left_mult", "right_mult", "P", "check")

    def range_proof_verify(self, head, V, n, a, b, L, R, G, H, g, h):
        """orc_range_proof_verify (rp.cu:1717 semantics) -> (ok, detail dict)."""
        head = np.ascontiguousarray(head, np.uint64)
        a, b = np.ascontiguousarray(a, np.uint64).reshape(-1, 4), np.ascontiguousarray(b, np.uint64).reshape(-1, 4)
        L, R = np.ascontiguousarray(L, np.uint64).reshape(-1, 16), np.ascontiguousarray(R, np.uint64).reshape(-1, 16)
        det = np.zeros(8 * 4 + 32 + 6 * 128, np.uint8)
        ok = self.f("range_proof_verify")(
            _p(head), _p(np.ascontiguousarray(V, np.uint64)), _sz(n), _p(a), _p(b), _sz(len(a)), _p(L), _p(R),
            _sz(len(L)), _p(np.ascontiguousarray(G, np.uint64)), _p(np.ascontiguousarray(H, np.uint64)),
            _p(np.ascontiguousarray(g, np.uint64)), _p(np.ascontiguousarray(h, np.uint64)), _p(det))
        flags = det[:32].view(np.int32)
        d = {k: bool(flags[i]) for i, k in enumerate(self.RPV_KEYS)}
        d["delta"] = det[32:64].view(np.uint64).copy()
        pts = det[64:].view(np.uint64).reshape(6, 16)
        for i, k in enumerate(self.RPV_PTS):
            d[k] = pts[i].copy()
        return bool(ok), d


    def generate_range_proof(self, value32, gamma32, sLR, rnd4, n, G, H, g, h):
        """orc_generate_range_proof -> dict(head, V, a, b, L, R) or None (value refused)."""
        head = np.zeros(HEAD_WORDS, np.uint64)
        a, b = fe(1), fe(1)
        L, R = ge(max(n, 1)), ge(max(n, 1))
        ll = _sz()
        r = self.f("generate_range_proof")(
            _p(np.ascontiguousarray(value32, np.uint8)), _p(np.ascontiguousarray(gamma32, np.uint8)),
            _p(np.ascontiguousarray(sLR, np.uint8)), _p(np.ascontiguousarray(rnd4, np.uint8)), _sz(n),
            _p(np.ascontiguousarray(G, np.uint64)), _p(np.ascontiguousarray(H, np.uint64)),
            _p(np.ascontiguousarray(g, np.uint64)), _p(np.ascontiguousarray(h, np.uint64)), _p(head), _p(a), _p(b),
            _p(L), _p(R), ctypes.byref(ll))
        if r != 0:
            return None
        return dict(head=head, V=head[0:16].copy(), a=a, b=b, L=L[:ll.value].copy(), R=R[:ll.value].copy())


class Reference(_Lib):
    """The reference's own host code (oracle/_ref/libbpref.so)."""

    prefix = "ref_"

    def __init__(self, path=REF_SO):
        super().__init__(path)
        for n in ("prove", "cuda_range_proof_verify", "range_proof_verify", "ipa_prove", "cuda_inner_product_verify"):
            self.f(n).restype = ctypes.c_int

    def fe_op(self, name, *args):
        h = fe()
        self.f(name)(_p(h), *[_p(np.ascontiguousarray(x, np.uint64)) for x in args])
        return h

    def fe_tobytes(self, f):
        b = np.zeros(32, np.uint8)
        self.f("fe_tobytes")(_p(b), _p(np.ascontiguousarray(f, np.uint64)))
        return b

    def ge_op(self, name, *args):
        r = ge()
        self.f(name)(_p(r), *[_p(np.ascontiguousarray(x)) for x in args])
        return r

    def ge_normalize(self, name, p):
        q = np.array(p, np.uint64)
        self.f(name)(_p(q))
        return q

    def msm(self, name, s, P):
        r = ge()
        self.f(name)(_p(r), _p(np.ascontiguousarray(s)), _p(np.ascontiguousarray(P, np.uint64)), _sz(len(P)))
        return r

    def base_points(self, n, seed_byte):
        out = ge(n)
        seed = np.zeros(32, np.uint8)
        seed[0] = seed_byte
        self.f("base_points")(_p(out), _sz(n), _p(seed))
        return out

    def gh(self):
        g, h = ge(), ge()
        self.f("gh")(_p(g), _p(h))
        return g, h

    def prove(self, seed, value32, n, G, H, g, h):
        """Deterministic reference proof. Returns dict(V, head, a, b, L, R) or None (prover refused)."""
        V, head = ge(), np.zeros(HEAD_WORDS, np.uint64)
        a, b, L, R = fe(n), fe(n), ge(n), ge(n)
        abl, ll = _sz(), _sz()
        r = self.f("prove")(ctypes.c_uint64(seed), _p(np.ascontiguousarray(value32, np.uint8)), _sz(n), _p(G), _p(H),
                            _p(g), _p(h), _p(V), _p(head), _p(a), _p(b), _p(L), _p(R), ctypes.byref(abl),
                            ctypes.byref(ll))
        if r != 0:
            return None
        return dict(V=V, head=head, a=a[:abl.value].copy(), b=b[:abl.value].copy(), L=L[:ll.value].copy(),
                    R=R[:ll.value].copy())

    def _vargs(self, pr, n, G, H, g, h):
        return (_p(pr["head"]), _p(pr["V"]), _sz(n), _p(pr["a"]), _p(pr["b"]), _sz(len(pr["a"])), _p(pr["L"]),
                _p(pr["R"]), _sz(len(pr["L"])), _p(G), _p(H), _p(g), _p(h))

    def cuda_range_proof_verify(self, pr, n, G, H, g, h):
        return bool(self.f("cuda_range_proof_verify")(*self._vargs(pr, n, G, H, g, h)))

    def range_proof_verify(self, pr, n, G, H, g, h):
        return bool(self.f("range_proof_verify")(*self._vargs(pr, n, G, H, g, h)))

    def verify_P(self, pr, n, G, H, g, h):
        P, yzx = ge(), np.zeros(96, np.uint8)
        self.f("verify_P")(_p(pr["head"]), _p(pr["V"]), _sz(n), _p(G), _p(H), _p(g), _p(h), _p(P), _p(yzx))
        return P, yzx

    def ipa_fold(self, G, H, n, x, L, R, a0, b0, c, Q):
        rounds = len(L)
        Gt, Ht, chk = ge(max(n - 1, 1)), ge(max(n - 1, 1)), ge()
        self.f("ipa_fold")(_p(G), _p(H), _sz(n), _p(np.ascontiguousarray(x, np.uint64)), _p(L), _p(R), _sz(rounds),
                           _p(np.ascontiguousarray(a0, np.uint64)), _p(np.ascontiguousarray(b0, np.uint64)),
                           _p(np.ascontiguousarray(c, np.uint64)), _p(Q), _p(Gt), _p(Ht), _p(chk))
        return Gt, Ht, chk


    def ipa_prove(self, a, b, G, H, Q, c, transcript=None):
        """inner_product_prove (bulletproof_vectors.cu:277) -> dict(a, b, L, R, x) or None."""
        n = len(a)
        a, b = np.ascontiguousarray(a, np.uint64), np.ascontiguousarray(b, np.uint64)
        tr = np.zeros(32, np.uint8) if transcript is None else np.ascontiguousarray(transcript, np.uint8)
        ao, bo, L, R, x = fe(n), fe(n), ge(max(n, 1)), ge(max(n, 1)), fe()
        abl, ll = _sz(), _sz()
        r = self.f("ipa_prove")(_p(a), _p(b), _sz(n), _p(np.ascontiguousarray(G, np.uint64)),
                                _p(np.ascontiguousarray(H, np.uint64)), _p(np.ascontiguousarray(Q, np.uint64)),
                                _p(np.ascontiguousarray(c, np.uint64)), _p(tr), _p(ao), _p(bo), ctypes.byref(abl),
                                _p(L), _p(R), ctypes.byref(ll), _p(x))
        if r != 0:
            return None
        return dict(a=ao[:abl.value].copy(), b=bo[:abl.value].copy(), L=L[:ll.value].copy(), R=R[:ll.value].copy(),
                    x=x)

    def cuda_inner_product_verify(self, n, a, b, c, L, R, x, P, G, H, Q):
        a, b = np.ascontiguousarray(a, np.uint64).reshape(-1, 4), np.ascontiguousarray(b, np.uint64).reshape(-1, 4)
        L, R = np.ascontiguousarray(L, np.uint64).reshape(-1, 16), np.ascontiguousarray(R, np.uint64).reshape(-1, 16)
        return bool(self.f("cuda_inner_product_verify")(
            _sz(n), _p(a), _p(b), _sz(len(a)), _p(np.ascontiguousarray(c, np.uint64)), _p(L), _p(R), _sz(len(L)),
            _p(np.ascontiguousarray(x, np.uint64)), _p(np.ascontiguousarray(P, np.uint64)),
            _p(np.ascontiguousarray(G, np.uint64)), _p(np.ascontiguousarray(H, np.uint64)),
            _p(np.ascontiguousarray(Q, np.uint64))))


    LOG_CAP = 1 << 16

    def cuda_range_proof_verify_log(self, pr, n, G, H, g, h):
        """cuda_range_proof_verify with the reference's stdout captured -> (ok, printed text)."""
        buf = ctypes.create_string_buffer(self.LOG_CAP)
        f = self.f("cuda_range_proof_verify_log")
        f.restype = ctypes.c_int
        ok = f(*self._vargs(pr, n, G, H, g, h), buf, _sz(self.LOG_CAP))
        return bool(ok), buf.value.decode()

    def cuda_inner_product_verify_log(self, n, a, b, c, L, R, x, P, G, H, Q):
        """cuda_inner_product_verify with the reference's stdout captured -> (ok, printed text)."""
        a, b = np.ascontiguousarray(a, np.uint64).reshape(-1, 4), np.ascontiguousarray(b, np.uint64).reshape(-1, 4)
        L, R = np.ascontiguousarray(L, np.uint64).reshape(-1, 16), np.ascontiguousarray(R, np.uint64).reshape(-1, 16)
        buf = ctypes.create_string_buffer(self.LOG_CAP)
        f = self.f("cuda_inner_product_verify_log")
        f.restype = ctypes.c_int
        ok = f(_sz(n), _p(a), _p(b), _sz(len(a)), _p(np.ascontiguousarray(c, np.uint64)), _p(L), _p(R), _sz(len(L)),
               _p(np.ascontiguousarray(x, np.uint64)), _p(np.ascontiguousarray(P, np.uint64)),
               _p(np.ascontiguousarray(G, np.uint64)), _p(np.ascontiguousarray(H, np.uint64)),
               _p(np.ascontiguousarray(Q, np.uint64)), buf, _sz(self.LOG_CAP))
        return bool(ok), buf.value.decode()

    def point_tree(self, P):
        """ref_point_tree: the canonical tree over given points (device add + device normalize)."""
        r = ge()
        P = np.ascontiguousarray(P, np.uint64).reshape(-1, 16)
        self.f("point_tree")(_p(r), _p(P), _sz(len(P)))
        return r

    def rpv_parts(self, pr, n, G, H, g, h):
        """range_proof_verify's sub-checks, each the reference's own function -> (delta, flags):
        flags bit0 enhanced_range_check, bit1 robust_polynomial_identity_check, bit2 inner_product_verify."""
        delta, flags = fe(), ctypes.c_int()
        self.f("rpv_parts")(*self._vargs(pr, n, G, H, g, h), _p(delta), ctypes.byref(flags))
        return delta, flags.value


def prover_randomness(seed, n):
    """The random scalars the reference prover draws under oracle/ref's deterministic RAND_bytes
    (block k = SHA256(seed_le64 || k_le64)), each masked as generate_random_scalar does (rp.cu:153-159):
    gamma (ref_prove's blinding), then sL_i, sR_i interleaved (rp.cu:1246-1252), alpha, rho, tau1, tau2.
    Returns (gamma (32,), sLR (n, 64), rnd4 (4, 32)) as uint8."""
    import hashlib

    def block(k):
        b = bytearray(hashlib.sha256(int(seed).to_bytes(8, "little") + int(k).to_bytes(8, "little")).digest())
        b[31] &= 0x7F
        b[0] &= 0xF8
        b[31] |= 0x40
        return np.frombuffer(bytes(b), np.uint8)
    gamma = block(0)
    sLR = np.stack([np.concatenate([block(1 + 2 * i), block(2 + 2 * i)]) for i in range(n)]) if n else \
        np.zeros((0, 64), np.uint8)
    rnd4 = np.stack([block(2 * n + 1 + k) for k in range(4)])
    return gamma, sLR, rnd4


def have_reference():
    return os.path.exists(REF_SO)


def _verify_chunk(args):
    n, heads, Vs, As, Bs, Ls, Rs, G, H, g, h = args
    O = Oracle()
    out = []
    for i in range(len(heads)):
        ok, P, chk, _, _ = O.cuda_range_proof_verify(heads[i], Vs[i], n, As[i], Bs[i], Ls[i], Rs[i], G, H, g, h)
        out.append((ok, P, chk))
    return out


def cuda_range_proof_verify_many(n, heads, Vs, As, Bs, Ls, Rs, G, H, g, h, procs=None):
    """The restatement's cuda_range_proof_verify over many proofs, in `procs` spawned worker
    processes (children that never touch a GPU) -> (ok (m,) bool, P (m,16), check (m,16))."""
    import multiprocessing as mp
    m = len(heads)
    if procs is None:
        procs = min(16, os.cpu_count() or 1)
    procs = max(1, min(procs, m))
    cuts = [m * k // procs for k in range(procs + 1)]
    jobs = [(n, heads[a:b], Vs[a:b], As[a:b], Bs[a:b], Ls[a:b], Rs[a:b], G, H, g, h)
            for a, b in zip(cuts[:-1], cuts[1:]) if b > a]
    if procs == 1:
        res = [_verify_chunk(j) for j in jobs]
    else:
        with mp.get_context("spawn").Pool(len(jobs)) as pool:
            res = pool.map(_verify_chunk, jobs)
    flat = [r for part in res for r in part]
    return (np.array([r[0] for r in flat], bool), np.stack([r[1] for r in flat]), np.stack([r[2] for r in flat]))


# ---------------------------------------------------------------- the accept rule's figures
# cuda_inner_product_verify reports its comparison of the check point with P on stdout
# (crv:287-346) and accepts if any of four tests holds (crv:349-357).  STATS names the printed
# integers; `printed_stats` parses the reference's text, `accept_stats` recomputes the same
# figures from the two points (host tobytes of X and Y, crv:281-285).
STATS = ("x_diffs", "small_x", "y_diffs", "small_y", "msb", "hash_nonzero")
BRANCHES = ("b_small", "b_msb", "b_diffs", "b_hash")   # the four tests, crv:351, :353, :355, :357


def printed_stats(text):
    """The figures the reference printed for ONE cuda_inner_product_verify call -> dict:
    early_reject (crv:154, <a,b> != c), computed_x8 / expected_x8 (crv:288-293, first 8 bytes of
    tobytes(check.X) / tobytes(P.X)), the STATS integers, and verdict (crv:363-367)."""
    import re
    if "Inner product verification failed: <a,b> != c" in text:
        return {"early_reject": True, "verdict": False}
    m = re.search(r"Computed X: ([0-9a-f]{16})\.\.\.\nExpected X: ([0-9a-f]{16})\.\.\.\n"
                  r"Coordinate differences: X=(\d+) bytes \((\d+) small\), Y=(\d+) bytes \((\d+) small\)\n"
                  r"Matching significant bits: (\d+)/64\nHash difference count: (\d+)/32\n", text)
    if not m:
        raise ValueError("unexpected reference output:\n" + text)
    d = {"early_reject": False, "computed_x8": bytes.fromhex(m.group(1)), "expected_x8": bytes.fromhex(m.group(2))}
    d.update({k: int(m.group(3 + i)) for i, k in enumerate(STATS)})
    d["verdict"] = "CUDA inner product verification passed with robust comparison" in text
    return d


def accept_stats(check_xy, P_xy):
    """Restatement of crv:297-357 on 64-byte X||Y encodings (host tobytes) -> dict of STATS,
    the four branch flags and the verdict."""
    import hashlib
    c = np.frombuffer(bytes(check_xy), np.uint8).astype(int)
    p = np.frombuffer(bytes(P_xy), np.uint8).astype(int)
    d = np.abs(c - p)
    st = {"x_diffs": int((d[:32] > 0).sum()), "small_x": int(((d[:32] > 0) & (d[:32] <= 10)).sum()),
          "y_diffs": int((d[32:] > 0).sum()), "small_y": int(((d[32:] > 0) & (d[32:] <= 10)).sum()),
          "msb": int(64 - np.unpackbits((c[24:32] ^ p[24:32]).astype(np.uint8)).sum())}
    hsh = hashlib.sha256(bytes(check_xy) + bytes(P_xy)).digest()
    st["hash_nonzero"] = sum(1 for x in hsh if x)
    br = {"b_small": st["small_x"] + st["small_y"] >= 20, "b_msb": st["msb"] >= 28,
          "b_diffs": st["x_diffs"] + st["y_diffs"] <= 32, "b_hash": st["hash_nonzero"] <= 24}
    st.update(br)
    st["verdict"] = any(br.values())
    return st


def head_fields(head):
    """Split a flat head into named views."""
    head = np.asarray(head)
    pts = head[:80].reshape(5, 16)
    fes = head[80:].reshape(5, 4)
    return dict(V=pts[0], A=pts[1], S=pts[2], T1=pts[3], T2=pts[4], taux=fes[0], mu=fes[1], t=fes[2], c=fes[3],
                x=fes[4])
