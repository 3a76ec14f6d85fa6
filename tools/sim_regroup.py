"""Cost model of phase-regrouped waves for the canonical MSM's per-lane scalar-mults (k_msm_points),
against the unified loop it would replace (VERDICT r05 ask 2; not a test).

Unified (today): every step is one ge25519_add(r, q) with q in {r, P} per lane, 1639 VALU
(tools/isa_count.py); lanes sorted by chain length, a wave runs as long as its longest lane.
Regrouped: every g scalar bits, a block's lanes are re-sorted by their next g-bit pattern (through
LDS), and each wave runs per bit one doubling (ge_dbl, 1475 VALU) and the Z2 = 1 add (1464) if any
of its lanes has that bit set.  The exchange itself (LDS traffic, ranks, barriers) is NOT counted:
the printed ratio is an upper bound of the gain.

  python tools/sim_regroup.py   (output: profiles/ab/r06a_msm_regroup_model.txt)
"""
import numpy as np

DBL, ADD, UNI = 1475, 1464, 1639


def unified_cost(bits, W=64):
    steps = []
    for b in bits:
        nz = np.flatnonzero(b)
        top = nz[0] if len(nz) else 256
        steps.append((256 - top) + b[top:].sum())
    steps = np.sort(np.array(steps))[::-1]
    return steps.reshape(-1, W).max(axis=1).sum() * UNI / (len(steps) // W)


def regroup_cost(bits, block, g, W=64):
    tot = 0
    for b0 in range(0, bits.shape[0], block):
        blk = bits[b0:b0 + block]
        for s in range(0, 256 - 256 % g, g):
            pat = blk[:, s:s + g]
            key = (pat * (1 << np.arange(g)[::-1])).sum(1)
            srt = pat[np.argsort(key, kind="stable")]
            for w in range(0, block, W):
                wp = srt[w:w + W]
                for j in range(g):
                    tot += DBL + (ADD if wp[:, j].any() else 0)
    return tot / (bits.shape[0] // W)


def main():
    rng = np.random.default_rng(1)
    bits = rng.integers(0, 2, size=(4096, 256))
    bits[:, 0] = 1
    u = unified_cost(bits)
    print(f"unified loop: {u:.0f} VALU per wave (4096 random full-length scalars)")
    print("block  g  regrouped  ratio (exchange cost not counted)")
    for block in (256, 512, 1024):
        for g in (1, 2, 4):
            r = regroup_cost(bits, block, g)
            print(f"{block:5d} {g:2d} {r:10.0f}  {r / u:.3f}")


if __name__ == "__main__":
    main()
