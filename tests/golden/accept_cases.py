"""The range-mode cases of tests/golden/accept_n*.npz (written by make_golden.py accept):
24 reference proofs stored whole, 168 tampered copies stored as (base proof, field, word, XOR
mask), 64 proof-shaped random inputs stored whole.  Shared by the generator and the tests."""
import numpy as np

TAMPER_FIELDS = ("head", "Varg", "a", "b", "L", "R")


def apply_tamper(pr, field, word, mask):
    """A copy of proof dict `pr` with word `word` of field TAMPER_FIELDS[field] XOR `mask`."""
    q = {k: np.array(v, np.uint64) for k, v in pr.items()}
    key = {0: "head", 1: "V"}.get(int(field), TAMPER_FIELDS[int(field)])
    flat = q[key].reshape(-1)
    flat[int(word)] ^= np.uint64(mask)
    return q


def accept_cases(d):
    """Rebuild the 256 range-mode case proofs of an accept_n*.npz fixture (dicts as R.prove returns)."""
    base = [dict(head=d["base_head"][i], V=d["base_V"][i], a=d["base_a"][i], b=d["base_b"][i], L=d["base_L"][i],
                 R=d["base_R"][i]) for i in range(len(d["base_head"]))]
    tam = [apply_tamper(base[int(b)], f, w, m) for (b, f, w), m in zip(d["tamper"], d["tamper_mask"])]
    rnd = [dict(head=d["rand_head"][i], V=d["rand_head"][i][0:16].copy(), a=d["rand_head"][i][88:92][None].copy(),
                b=np.array([[1, 0, 0, 0]], np.uint64), L=d["rand_L"][i], R=d["rand_R"][i])
           for i in range(len(d["rand_head"]))]
    return base + tam + rnd
