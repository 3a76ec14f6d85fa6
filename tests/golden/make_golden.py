"""Generate the golden fixtures in tests/golden/ from the REFERENCE ITSELF.

Run in the build container (needs /root/reference):  python tests/golden/make_golden.py
It builds oracle/_ref/libbpref.so (the reference's host sources compiled in place by
oracle/build_ref.sh) and records inputs + reference outputs as .npz (no pickles):

  field.npz   edge-heavy pairs -> fe25519_add/sub/mul/invert/tobytes      (curve25519_ops.cu:41-251)
  point.npz   ge25519_add, host/device normalize, scalarmult               (curve25519_ops.cu:326-605, .cuh:188-290)
  msm.npz     canonical-tree GPU MSM semantics + CPU MSM, n in {1,2,3,5,16,17,64}
  proofs_n16.npz / proofs_n64.npz
              reference proofs (generate_range_proof, deterministic RAND), the verdicts of
              cuda_range_proof_verify and range_proof_verify, P (calculate_inner_product_point),
              the IPA fold trace and the check point (crv:160-279 composed from reference primitives)
  ipa4096.npz BASELINE configs[3]: inner_product_prove (bulletproof_vectors.cu:277)
              at n = 4096 on SHA-derived a, b (ipa_vectors below), G/H = base points {1}/{2}, Q = h,
              transcript 0^32; P = canonical-tree GPU-MSM semantics over (a||b, G||H).  The prover keeps
              c = c_in, and with this arithmetic <a',b'> != c_in, so cuda_inner_product_verify would reject
              at crv:146-158 before folding (recorded as ok_raw); the fold case sets c = <a',b'> (c_fix).
              Recorded: the verdicts, the check point and the last 15 folded G'/H' (rounds 9-11).

  rpverify.npz range_proof_verify (bulletproof_range_proof.cu:1717) on reference proofs,
              tampered copies (V argument != proof V, t / taux / mu / c perturbed) and proof-shaped
              random inputs, n in {16, 64}: the verdict and, from the reference's own functions,
              compute_precise_delta's delta and the enhanced_range_check /
              robust_polynomial_identity_check / inner_product_verify results.

  batch1024.npz BASELINE configs[1] at full batch: 1024 reference proofs of random 64-bit values
              + 256 tampered copies, the reference's cuda_range_proof_verify outcome of each
              (verdict, early reject, 8-byte digests of the proof, P and the check point).

  python tests/golden/make_golden.py [ipa4096|rpverify|accept|printed|batch1024]
              (argument: regenerate only that fixture)

The survey's golden digests are reproduced by tests/test_oracle_golden.py.
"""
import hashlib
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
from oracle import pyoracle as po  # noqa: E402
from accept_cases import TAMPER_FIELDS, apply_tamper  # noqa: E402

M = 2**64 - 1
P = [0xFFFFFFFFFFFFFFED, M, M, 0x7FFFFFFFFFFFFFFF]
EDGE = [0, 1, 2, 3, 19, 38, M, M - 1, M - 18, M - 19, M - 20, 2**63, 2**63 - 1, 2**63 + 1, 2**32, 2**32 - 1,
        P[0] - 1, P[0] + 1]


def edge_fe(rng, k):
    out = np.zeros((k, 4), np.uint64)
    for i in range(k):
        mode = rng.integers(0, 4)
        for j in range(4):
            if mode == 0 or rng.random() < 0.3:
                out[i, j] = np.uint64(int(rng.integers(0, 2**63)) * 2 + int(rng.integers(0, 2)))
            else:
                out[i, j] = np.uint64(EDGE[rng.integers(0, len(EDGE))])
    # a few exact multiples/near-multiples of p
    special = [P, [P[0] + 1, M, M, P[3]], [M, M, M, M], [P[0] - 1, M, M, P[3]]]
    for i in range(min(k, len(special)) if k >= 8 else 0):
        out[i] = special[i]
    return out


def main():
    po.build()
    R = po.Reference()
    rng = np.random.default_rng(20251015)

    # ---------------------------------------------------------------- field
    k = 256
    f, g = edge_fe(rng, k), edge_fe(rng, k)
    res = {n: np.zeros((k, 4), np.uint64) for n in ("add", "sub", "mul", "invert")}
    tob = np.zeros((k, 32), np.uint8)
    for i in range(k):
        res["add"][i] = R.fe_op("fe_add", f[i], g[i])
        res["sub"][i] = R.fe_op("fe_sub", f[i], g[i])
        res["mul"][i] = R.fe_op("fe_mul", f[i], g[i])
        res["invert"][i] = R.fe_op("fe_invert", f[i])
        tob[i] = R.fe_tobytes(f[i])
    np.savez_compressed(os.path.join(HERE, "field.npz"), f=f, g=g, tobytes=tob, **res)

    # ---------------------------------------------------------------- points
    kp = 48
    p = np.concatenate([edge_fe(rng, kp), edge_fe(rng, kp), edge_fe(rng, kp), edge_fe(rng, kp)], axis=1)
    q = np.concatenate([edge_fe(rng, kp), edge_fe(rng, kp), edge_fe(rng, kp), edge_fe(rng, kp)], axis=1)
    base = R.base_points(8, 9)
    p[:8] = base
    add = np.stack([R.ge_op("ge_add", p[i], q[i]) for i in range(kp)])
    nh = np.stack([R.ge_normalize("ge_normalize", p[i]) for i in range(kp)])
    nd = np.stack([R.ge_normalize("dev_ge_normalize", p[i]) for i in range(kp)])
    ks = 12
    sc = rng.integers(0, 256, size=(ks, 32)).astype(np.uint8)
    sc[0] = 0
    sc[1] = 0
    sc[1, 0] = 1
    sc[2] = 255
    sc[3] = 0
    sc[3, 5] = 42
    sm = np.stack([R.ge_op("ge_scalarmult", sc[i], p[i]) for i in range(ks)])
    np.savez_compressed(os.path.join(HERE, "point.npz"), p=p, q=q, add=add, norm_host=nh, norm_dev=nd,
                        scalars=sc, scalarmult=sm)

    # ---------------------------------------------------------------- MSM
    out = {}
    for n in (1, 2, 3, 5, 16, 17, 64):
        Pn = R.base_points(n, 5)
        s = edge_fe(rng, n) if n != 64 else np.stack(
            [np.frombuffer(hashlib.sha256(b"msm-s" + i.to_bytes(4, "little")).digest(), "<u8") for i in range(n)])
        if n == 64:
            s = s.astype(np.uint64)
            s[:, 3] &= np.uint64(0x7FFFFFFFFFFFFFFF)
        out[f"P{n}"] = Pn
        out[f"s{n}"] = s
        out[f"canon{n}"] = R.msm("msm_canon", s, Pn)
        out[f"cpu{n}"] = R.msm("msm_cpu", s, Pn)
    np.savez_compressed(os.path.join(HERE, "msm.npz"), **out)

    # ---------------------------------------------------------------- proofs
    for n in (16, 64):
        G, H = R.base_points(n, 1), R.base_points(n, 2)
        g, h = R.gh()
        recs = dict(G=G, H=H, g=g, h=h)
        heads, Vs, As, Bs, Ls, Rs, oks, okc, Ps, chks, Gts, Hts, vals = ([] for _ in range(13))
        for seed in range(1, 7):
            val = np.zeros(32, np.uint8)
            if seed == 1:
                val[0] = 42                      # complete_bulletproof_test.cu:116
            else:
                val[:n // 8] = rng.integers(0, 256, n // 8)
            pr = R.prove(seed, val, n, G, H, g, h)
            hd = po.head_fields(pr["head"])
            Pr, _ = R.verify_P(pr, n, G, H, g, h)
            Gt, Ht, chk = R.ipa_fold(G, H, n, hd["x"], pr["L"], pr["R"], pr["a"][0], pr["b"][0], hd["c"], h)
            heads.append(pr["head"]); Vs.append(pr["V"]); As.append(pr["a"]); Bs.append(pr["b"])
            Ls.append(pr["L"]); Rs.append(pr["R"]); vals.append(val)
            oks.append(R.cuda_range_proof_verify(pr, n, G, H, g, h))
            okc.append(R.range_proof_verify(pr, n, G, H, g, h))
            Ps.append(Pr); chks.append(chk); Gts.append(Gt); Hts.append(Ht)
        np.savez_compressed(os.path.join(HERE, f"proofs_n{n}.npz"), **recs, head=np.stack(heads), V=np.stack(Vs),
                            a=np.stack(As), b=np.stack(Bs), L=np.stack(Ls), R=np.stack(Rs), value=np.stack(vals),
                            ok_cuda=np.array(oks), ok_cpu=np.array(okc), P=np.stack(Ps), check=np.stack(chks),
                            Gtrace=np.stack(Gts), Htrace=np.stack(Hts))
    print("fixtures written to", HERE)


def ipa_vectors(n):
    """a_i = SHA256("ipa-a" || i_le32), b_i = SHA256("ipa-b" || i_le32), byte 31 &= 0x7F, LE limbs."""
    def vec(tag):
        v = np.stack([np.frombuffer(hashlib.sha256(tag + i.to_bytes(4, "little")).digest(), "<u8")
                      for i in range(n)]).astype(np.uint64)
        v[:, 3] &= np.uint64(0x7FFFFFFFFFFFFFFF)
        return v
    return vec(b"ipa-a"), vec(b"ipa-b")


def make_ipa4096():
    po.build()
    R = po.Reference()
    n = 4096
    a, b = ipa_vectors(n)
    G, H = R.base_points(n, 1), R.base_points(n, 2)
    _, Q = R.gh()
    c_in = po.fe()
    R.f("inner_product")(po._p(c_in), po._p(a), po._p(b), po._sz(n))
    pr = R.ipa_prove(a, b, G, H, Q, c_in)
    c_fix = po.fe()
    R.f("inner_product")(po._p(c_fix), po._p(pr["a"]), po._p(pr["b"]), po._sz(len(pr["a"])))
    P = R.msm("msm_canon", np.concatenate([a, b]), np.concatenate([G, H]))
    ok_raw = R.cuda_inner_product_verify(n, pr["a"], pr["b"], c_in, pr["L"], pr["R"], pr["x"], P, G, H, Q)
    ok = R.cuda_inner_product_verify(n, pr["a"], pr["b"], c_fix, pr["L"], pr["R"], pr["x"], P, G, H, Q)
    Gt, Ht, chk = R.ipa_fold(G, H, n, pr["x"], pr["L"], pr["R"], pr["a"][0], pr["b"][0], c_fix, Q)
    np.savez_compressed(os.path.join(HERE, "ipa4096.npz"), n=np.array(n), c_in=c_in, c_fix=c_fix, a=pr["a"],
                        b=pr["b"], L=pr["L"], R=pr["R"], x=pr["x"], P=P, ok=np.array(ok), ok_raw=np.array(ok_raw),
                        check=chk, Gtail=Gt[-15:], Htail=Ht[-15:])
    print("ipa4096: ok", ok, "ok_raw", ok_raw)


def make_rpverify():
    po.build()
    R = po.Reference()
    rng = np.random.default_rng(77)
    out = {}
    for n, nproofs in ((16, 4), (64, 2)):
        G, H = R.base_points(n, 1), R.base_points(n, 2)
        g, h = R.gh()
        cases = []
        for seed in range(101, 101 + nproofs):
            val = np.zeros(32, np.uint8)
            val[:n // 8] = rng.integers(0, 256, n // 8)
            pr = R.prove(seed, val, n, G, H, g, h)
            cases.append(("ref", pr))
            for kind, word in (("t", 90), ("taux", 80), ("mu", 84), ("c", 92)):
                q = {k: v.copy() for k, v in pr.items()}
                q["head"][word] ^= np.uint64(1 << int(rng.integers(0, 60)))
                cases.append((kind, q))
            q = {k: v.copy() for k, v in pr.items()}
            q["V"][0] ^= np.uint64(1)                 # V argument != proof.V (rp.cu:1735)
            cases.append(("V", q))
        for _ in range(4):                            # proof-shaped random inputs
            hd = np.zeros(po.HEAD_WORDS, np.uint64)
            hd[:] = rng.integers(0, 2**63, po.HEAD_WORDS, dtype=np.uint64)
            pr = dict(head=hd, V=hd[0:16].copy(), a=hd[88:92][None].copy(), b=np.array([[1, 0, 0, 0]], np.uint64),
                      L=rng.integers(0, 2**63, (n.bit_length() - 1, 16), dtype=np.uint64),
                      R=rng.integers(0, 2**63, (n.bit_length() - 1, 16), dtype=np.uint64))
            pr["head"][92:96] = pr["head"][88:92]     # c = t = <[t],[1]>
            cases.append(("rand", pr))
        recs = {k: [] for k in ("kind", "head", "V", "a", "b", "L", "R", "ok", "delta", "flags")}
        for kind, pr in cases:
            recs["kind"].append(kind)
            for k in ("head", "V", "a", "b", "L", "R"):
                recs[k].append(pr[k])
            recs["ok"].append(R.range_proof_verify(pr, n, G, H, g, h))
            d, f = R.rpv_parts(pr, n, G, H, g, h)
            recs["delta"].append(d)
            recs["flags"].append(f)
        for k, v in recs.items():
            out[f"n{n}_{k}"] = np.array(v) if k == "kind" else np.stack([np.asarray(x) for x in v])
        print(f"rpverify n={n}: ok {sum(recs['ok'])}/{len(cases)}, flags {recs['flags']}")
    np.savez_compressed(os.path.join(HERE, "rpverify.npz"), **out)


# ---------------------------------------------------------------- accept_n16 / accept_n64
# cuda_range_proof_verify's tolerant accept rule (crv:297-357) pinned by the reference's OWN
# printed figures.  Per n, 256 range-mode cases:
#   * 24 reference proofs (seeds 201..224, random in-range values);
#   * 168 tampered copies: one 64-bit word of one field XOR-ed with a random mask (tamper_* below:
#     field code, flat word index, mask), 7 per reference proof, the kinds cycling through
#     TAMPER_KINDS (a / b / c tampering ends at the <a,b> != c early reject, crv:146-158; L[0] /
#     R[0] and taux / mu are never read by this verify);
#   * 64 proof-shaped random inputs (a = [t], b = [1], c = t).
# Recorded per case: the verdict, the reference's printed report (early reject flag, "Computed X"
# / "Expected X" 8 bytes, the six integers of crv:313-346: pyoracle.STATS), P from the reference's
# calculate_inner_product_point, the check point from ref_ipa_fold, and `check_pin`: the reference's
# report when it verifies the same inner-product proof against P := that check point (six zeros
# prove that the composed check point's X and Y bytes are the reference's own).
# Plus 32 IPA-level cases (cuda_inner_product_verify with a crafted P, 8 proofs x 4 variants)
# that reach the two branches no natural input reaches: the small-difference count (>= 20) and
# the differing-byte count (<= 32), each alone, next to "all equal" and a reject; the hash branch
# (<= 24 non-zero bytes of a SHA-256 output) is out of reach of any input (probability ~1e-12).
TAMPER_KINDS = (("L", 1), ("R", 1), ("x", 0), ("t", 0), ("A", 0), ("S", 0), ("T1", 0), ("T2", 0), ("a", 0),
                ("b", 0), ("c", 0), ("Varg", 0), ("L", 0), ("R", 0), ("taux", 0), ("mu", 0))
HEAD_OFF = {"V": 0, "A": 16, "S": 32, "T1": 48, "T2": 64, "taux": 80, "mu": 84, "t": 88, "c": 92, "x": 96}
def tamper_target(kind, sel, Lr, rng):
    """(field code, flat word index) for a tamper kind; sel = 1 picks a round >= 1 of L/R, 0 round 0."""
    if kind in HEAD_OFF:
        return 0, HEAD_OFF[kind] + int(rng.integers(0, 16 if kind in ("A", "S", "T1", "T2") else 4))
    if kind == "Varg":
        return 1, int(rng.integers(0, 16))
    if kind in ("a", "b"):
        return TAMPER_FIELDS.index(kind), int(rng.integers(0, 4))
    rnd = int(rng.integers(1, Lr)) if sel else 0
    return TAMPER_FIELDS.index(kind), rnd * 16 + int(rng.integers(0, 8))   # X or Y of L/R[rnd]


def _xy(O, p):
    return np.concatenate([O.fe_tobytes(p[0:4]), O.fe_tobytes(p[4:8])])


def _printed_row(st):
    """printed_stats dict -> (early, x8 computed, x8 expected, six ints) fixed-size arrays."""
    if st["early_reject"]:
        return 1, np.zeros(8, np.uint8), np.zeros(8, np.uint8), np.full(6, -1, np.int32)
    return (0, np.frombuffer(st["computed_x8"], np.uint8), np.frombuffer(st["expected_x8"], np.uint8),
            np.array([st[k] for k in po.STATS], np.int32))


def craft_P(O, chk, variant, rng):
    """A point whose X||Y host bytes sit at a chosen distance from the check point's (variant
    0: equal; 1: X bytes 24-31 flipped + >= 26 other bytes off by 1..3 (small count alone);
    2: X bytes 24-31 flipped only (differing-byte count alone); 3: X bytes 24-31 flipped + 30
    other bytes off by 0x80 (no test holds)).  Z = 1, T = the check point's (not compared)."""
    xy = _xy(O, chk).astype(np.int64)
    if variant:
        xy[24:31] ^= 0xFF
        xy[31] ^= 0x3F                       # bit 255 stays clear: the bytes stay a canonical encoding
    others = [i for i in range(63) if not 24 <= i < 32]   # never byte 63 (Y's top byte)
    pick = rng.permutation(others)
    if variant == 1:
        for i in pick[:27]:
            xy[i] = xy[i] + int(rng.integers(1, 4)) if xy[i] < 250 else xy[i] - int(rng.integers(1, 4))
    if variant == 3:
        for i in pick[:30]:
            xy[i] ^= 0x80
    b = xy.astype(np.uint8)
    P = np.zeros(16, np.uint64)
    P[0:4] = b[:32].view(np.uint64)
    P[4:8] = b[32:].view(np.uint64)
    P[8] = 1
    P[12:16] = chk[12:16]
    assert np.array_equal(_xy(O, P), b), "crafted bytes must be canonical"
    return P


def make_printed():
    """Add to proofs_n16/n64.npz and ipa4096.npz what the reference PRINTS about each check point
    (crv:287-346): printed_early, printed_x8c / printed_x8e ("Computed X" / "Expected X"),
    printed_stats (pyoracle.STATS), printed_ok; and check_pin, its report when the same proof is
    verified against P := the stored (composed) check point — six zeros pin every X / Y byte."""
    po.build()
    R = po.Reference()
    for n in (16, 64):
        path = os.path.join(HERE, f"proofs_n{n}.npz")
        d = dict(np.load(path))
        rows, pins, oks = [], [], []
        for i in range(len(d["head"])):
            pr = dict(head=d["head"][i], V=d["V"][i], a=d["a"][i], b=d["b"][i], L=d["L"][i], R=d["R"][i])
            ok, txt = R.cuda_range_proof_verify_log(pr, n, d["G"], d["H"], d["g"], d["h"])
            rows.append(_printed_row(po.printed_stats(txt)))
            oks.append(ok)
            hd = po.head_fields(pr["head"])
            _, t2 = R.cuda_inner_product_verify_log(n, pr["a"], pr["b"], hd["c"], pr["L"], pr["R"], hd["x"],
                                                    d["check"][i], d["G"], d["H"], d["h"])
            pins.append(_printed_row(po.printed_stats(t2))[3])
        d.update(printed_ok=np.array(oks), printed_early=np.array([r[0] for r in rows], np.uint8),
                 printed_x8c=np.stack([r[1] for r in rows]), printed_x8e=np.stack([r[2] for r in rows]),
                 printed_stats=np.stack([r[3] for r in rows]), check_pin=np.stack(pins))
        np.savez_compressed(path, **d)
        print(f"proofs_n{n}: printed stats {d['printed_stats'].tolist()}, pins {d['check_pin'].tolist()}")
    path = os.path.join(HERE, "ipa4096.npz")
    d = dict(np.load(path))
    n = int(d["n"])
    G, H = R.base_points(n, 1), R.base_points(n, 2)
    _, Q = R.gh()
    res = {}
    for tag, c, P in (("", d["c_fix"], d["P"]), ("_raw", d["c_in"], d["P"]), ("_pin", d["c_fix"], d["check"])):
        ok, txt = R.cuda_inner_product_verify_log(n, d["a"], d["b"], c, d["L"], d["R"], d["x"], P, G, H, Q)
        e, x8c, x8e, s6 = _printed_row(po.printed_stats(txt))
        res.update({f"printed_ok{tag}": np.array(ok), f"printed_early{tag}": np.array(e, np.uint8),
                    f"printed_x8c{tag}": x8c, f"printed_x8e{tag}": x8e, f"printed_stats{tag}": s6})
    d.update(res)
    np.savez_compressed(path, **d)
    print("ipa4096:", {k: v.tolist() for k, v in res.items() if "stats" in k or "ok" in k})


def make_accept():
    po.build()
    R = po.Reference()
    O = po.Oracle()
    for n in (16, 64):
        rng = np.random.default_rng(4000 + n)
        Lr = n.bit_length() - 1
        G, H = R.base_points(n, 1), R.base_points(n, 2)
        g, h = R.gh()
        base = []
        for seed in range(201, 225):
            val = np.zeros(32, np.uint8)
            val[:n // 8] = rng.integers(0, 256, n // 8)
            base.append(R.prove(seed, val, n, G, H, g, h))
        tam = []                                   # (base index, field, word, mask)
        for j in range(len(base) * 7):
            kind, sel = TAMPER_KINDS[j % len(TAMPER_KINDS)]
            f, w = tamper_target(kind, sel, Lr, rng)
            mask = 1 << int(rng.integers(0, 64)) if j % 2 else int(rng.integers(1, 2**63))
            tam.append((j // 7, f, w, mask))
        rnd = []
        for _ in range(64):
            hd = rng.integers(0, 2**63, po.HEAD_WORDS, dtype=np.uint64)
            hd[92:96] = hd[88:92]                  # c = t = <[t],[1]>
            rnd.append(dict(head=hd, V=hd[0:16].copy(), a=hd[88:92][None].copy(),
                            b=np.array([[1, 0, 0, 0]], np.uint64),
                            L=rng.integers(0, 2**63, (Lr, 16), dtype=np.uint64),
                            R=rng.integers(0, 2**63, (Lr, 16), dtype=np.uint64)))
        cases = [("ref", p) for p in base] + [("tamper", apply_tamper(base[b], f, w, m)) for b, f, w, m in tam] + \
                [("rand", p) for p in rnd]
        rec = {k: [] for k in ("ok", "early", "x8c", "x8e", "stats", "P", "check", "pin")}
        for kind, pr in cases:
            ok, txt = R.cuda_range_proof_verify_log(pr, n, G, H, g, h)
            st = po.printed_stats(txt)
            assert st["verdict"] == ok
            e, x8c, x8e, s6 = _printed_row(st)
            P, _ = R.verify_P(pr, n, G, H, g, h)
            hd = po.head_fields(pr["head"])
            _, _, chk = R.ipa_fold(G, H, n, hd["x"], pr["L"], pr["R"], pr["a"][0], pr["b"][0], hd["c"], h)
            pin = np.full(6, -1, np.int32)
            if not e:   # the composed check point against the reference's own: verify with P := it
                ok2, t2 = R.cuda_inner_product_verify_log(n, pr["a"], pr["b"], hd["c"], pr["L"], pr["R"], hd["x"], chk,
                                                          G, H, h)
                pin = _printed_row(po.printed_stats(t2))[3]
            for k, v in zip(rec, (ok, e, x8c, x8e, s6, P, chk, pin)):
                rec[k].append(v)
        # IPA-level crafted P: the branches natural inputs do not reach
        ipa = {k: [] for k in ("base", "variant", "P", "ok", "stats")}
        for b in range(8):
            pr = base[b]
            hd = po.head_fields(pr["head"])
            _, _, chk = R.ipa_fold(G, H, n, hd["x"], pr["L"], pr["R"], pr["a"][0], pr["b"][0], hd["c"], h)
            for v in range(4):
                Pc = craft_P(O, chk, v, rng)
                ok, txt = R.cuda_inner_product_verify_log(n, pr["a"], pr["b"], hd["c"], pr["L"], pr["R"], hd["x"], Pc,
                                                          G, H, h)
                st = po.printed_stats(txt)
                for k, val in zip(ipa, (b, v, Pc, ok, _printed_row(st)[3])):
                    ipa[k].append(val)
        out = dict(G=G, H=H, g=g, h=h,
                   base_head=np.stack([p["head"] for p in base]), base_V=np.stack([p["V"] for p in base]),
                   base_a=np.stack([p["a"] for p in base]), base_b=np.stack([p["b"] for p in base]),
                   base_L=np.stack([p["L"] for p in base]), base_R=np.stack([p["R"] for p in base]),
                   tamper=np.array([t[:3] for t in tam], np.int64),
                   tamper_mask=np.array([t[3] for t in tam], np.uint64),
                   rand_head=np.stack([p["head"] for p in rnd]), rand_L=np.stack([p["L"] for p in rnd]),
                   rand_R=np.stack([p["R"] for p in rnd]),
                   ok=np.array(rec["ok"]), early=np.array(rec["early"], np.uint8), x8c=np.stack(rec["x8c"]),
                   x8e=np.stack(rec["x8e"]), stats=np.stack(rec["stats"]), P=np.stack(rec["P"]),
                   check=np.stack(rec["check"]), check_pin=np.stack(rec["pin"]),
                   ipa_base=np.array(ipa["base"], np.int64), ipa_variant=np.array(ipa["variant"], np.int64),
                   ipa_P=np.stack(ipa["P"]), ipa_ok=np.array(ipa["ok"]), ipa_stats=np.stack(ipa["stats"]))
        np.savez_compressed(os.path.join(HERE, f"accept_n{n}.npz"), **out)
        print(f"accept n={n}: {len(cases)} cases, {int(out['ok'].sum())} accepts, {int(out['early'].sum())} early "
              f"rejects; ipa crafted ok {out['ipa_ok'].astype(int).tolist()}")


B1024_SEED0 = 5001   # seeds 5001 .. 6024 (disjoint from every other fixture's)


def batch1024_value(seed):
    """The 64-bit value of batch1024 proof `seed`: bytes 0..7 of SHA256("batch1024" || seed_le64)."""
    v = np.zeros(32, np.uint8)
    v[:8] = np.frombuffer(hashlib.sha256(b"batch1024" + int(seed).to_bytes(8, "little")).digest()[:8], np.uint8)
    return v


def proof_digest(pr):
    """8-byte SHA-256 of a proof's words (head, V, a, b, L, R): the GPU prover's reproduction check."""
    return hashlib.sha256(b"".join(np.ascontiguousarray(pr[k], np.uint64).tobytes()
                                   for k in ("head", "V", "a", "b", "L", "R"))).digest()[:8]


def point_digest(p):
    return hashlib.sha256(np.ascontiguousarray(p, np.uint64).tobytes()).digest()[:8]


def _b1024_rows(args):
    """Worker (spawned, no GPU): reference proofs / tampered copies -> per-case outcomes."""
    lo, hi, tam = args
    R = po.Reference()
    n = 64
    G, H = R.base_points(n, 1), R.base_points(n, 2)
    g, h = R.gh()
    out = []
    cache = {}

    def proof(i):
        if i not in cache:
            cache[i] = R.prove(B1024_SEED0 + i, batch1024_value(B1024_SEED0 + i), n, G, H, g, h)
        return cache[i]
    jobs = [(i, None) for i in range(lo, hi)] + [(t[0], t) for t in tam]
    for i, t in jobs:
        pr = proof(i) if t is None else apply_tamper(proof(i), *t[1:])
        ok, txt = R.cuda_range_proof_verify_log(pr, n, G, H, g, h)
        early = po.printed_stats(txt)["early_reject"]   # crv:146-158: <a,b> != c, no check point formed
        P, _ = R.verify_P(pr, n, G, H, g, h)
        hd = po.head_fields(pr["head"])
        _, _, chk = R.ipa_fold(G, H, n, hd["x"], pr["L"], pr["R"], pr["a"][0], pr["b"][0], hd["c"], h)
        out.append((i, t is not None, proof_digest(pr), bool(ok), point_digest(P), point_digest(chk), bool(early)))
    return out


def make_batch1024(procs=8):
    """BASELINE configs[1] at its full batch: 1024 reference proofs of random 64-bit values
    (generate_range_proof, rp.cu:1159, seeds 5001.. under oracle/ref's deterministic RAND_bytes)
    and 256 tampered copies (TAMPER_KINDS, one word XOR a mask), each verified by the reference's
    own cuda_range_proof_verify (crv:82-127).  Stored per case: the seed index, the value, 8-byte
    SHA-256 digests of the proof words, of P (calculate_inner_product_point) and of the check
    point (crv:160-279), and the reference's verdict -> batch1024.npz (no proof data: the GPU
    prover regenerates the proofs from seed and value, tests/test_gpu_fullsize.py)."""
    import multiprocessing as mp
    po.build()
    B, Lr = 1024, 6
    rng = np.random.default_rng(1024)
    tam = []
    for j in range(256):
        kind, sel = TAMPER_KINDS[j % len(TAMPER_KINDS)]
        f, w = tamper_target(kind, sel, Lr, rng)
        mask = 1 << int(rng.integers(0, 64)) if j % 2 else int(rng.integers(1, 2**63))
        tam.append((int(rng.integers(0, B)), f, w, mask))
    cuts = [B * k // procs for k in range(procs + 1)]
    jobs = [(cuts[k], cuts[k + 1], [t for t in tam if cuts[k] <= t[0] < cuts[k + 1]]) for k in range(procs)]
    with mp.get_context("spawn").Pool(procs) as pool:
        rows = [r for part in pool.map(_b1024_rows, jobs) for r in part]
    orig = sorted([r for r in rows if not r[1]], key=lambda r: r[0])
    tmap = {}
    for r in rows:
        if r[1]:
            tmap.setdefault(r[0], []).append(r)
    trows = []
    for t in tam:   # the tampered rows in `tam` order (a worker ran its share in that order)
        trows.append(tmap[t[0]].pop(0))
    cat = lambda rs, k: np.stack([np.frombuffer(r[k], np.uint8) for r in rs])
    out = dict(seed0=np.array(B1024_SEED0), value=np.stack([batch1024_value(B1024_SEED0 + i)[:8].view("<u8")[0]
                                                             for i in range(B)]).astype(np.uint64),
               proof_d8=cat(orig, 2), ok=np.array([r[3] for r in orig]), P_d8=cat(orig, 4), check_d8=cat(orig, 5),
               early=np.array([r[6] for r in orig]),
               tamper=np.array([t[:3] for t in tam], np.int64), tamper_mask=np.array([t[3] for t in tam], np.uint64),
               t_proof_d8=cat(trows, 2), t_ok=np.array([r[3] for r in trows]), t_P_d8=cat(trows, 4),
               t_check_d8=cat(trows, 5), t_early=np.array([r[6] for r in trows]))
    np.savez_compressed(os.path.join(HERE, "batch1024.npz"), **out)
    print(f"batch1024: {int(out['ok'].sum())}/{B} reference accepts, tampered {int(out['t_ok'].sum())}/256 accepts")


if __name__ == "__main__":
    if sys.argv[1:] == ["batch1024"]:
        make_batch1024()
    elif sys.argv[1:] == ["ipa4096"]:
        make_ipa4096()
    elif sys.argv[1:] == ["rpverify"]:
        make_rpverify()
    elif sys.argv[1:] == ["accept"]:
        make_accept()
    elif sys.argv[1:] == ["printed"]:
        make_printed()
    else:
        main()
        make_ipa4096()
        make_printed()
        make_rpverify()
        make_accept()
