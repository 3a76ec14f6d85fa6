"""Golden digest of the full-size configs[2] MSM (2^20 points), from the REFERENCE's own primitives.

Inputs exactly as SURVEY §8(d) config 3 / §8c: points = generate_deterministic_base_points
with seed {5} (complete_bulletproof_test.cu:33-63: SHA-256 derived X, Y, Z = 1, T = X*Y),
scalars_i = SHA256("msm-s" || i_le32) with byte 31 &= 0x7F.  Result = the canonical-tree MSM
(cuda_bulletproof_kernels.cu:26-207 as point_multi_scalar_mul_shared_kernel defines it).

The canonical tree decomposes exactly over aligned power-of-two shards, so the
2^20 scalar multiplications run as 8 shards of 2^17 in 8 processes, each through the reference
build's ref_msm_canon (oracle/_ref/libbpref.so: the reference's device_ge25519_scalarmult /
_add / _normalize from device_curve25519_ops.cuh compiled for the host, in the canonical order of
cuda_bulletproof_kernels.cu:141-168), and the 8 shard roots are combined by ref_point_tree (the
same tree levels).  The result is reference-emitted; the CPU restatement (oracle/bp_oracle.c)
computes the same bits (checked here: its shard roots and tree must agree).

    python tests/golden/make_msm_2p20.py      # ~2 min on 8 cores -> tests/golden/msm_2p20.json

It also records the Pippenger (window 12) result of the same inputs from orc_msm_pippenger: the
labelled alternative of include/cudabulletproof_hip.h hipbp_msm_pippenger (not the reference's
MSM bits; pinned to the C restatement of the bucket algorithm only).
"""
import hashlib
import json
import multiprocessing as mp
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

LOG2 = 20
SHARDS = 8


def scalars(n):
    s = np.stack([np.frombuffer(hashlib.sha256(b"msm-s" + i.to_bytes(4, "little")).digest(), "<u8")
                  for i in range(n)]).astype(np.uint64)
    s[:, 3] &= np.uint64(0x7FFFFFFFFFFFFFFF)
    return s


def _shard(k):
    from oracle import pyoracle
    R = pyoracle.Reference()
    n = 1 << LOG2
    m = n // SHARDS
    P = R.base_points(n, 5)[k * m:(k + 1) * m]
    s = scalars(n)[k * m:(k + 1) * m]
    return R.msm("msm_canon", s, P)


def _shard_oracle(k):
    from oracle import pyoracle
    O = pyoracle.Oracle()
    n = 1 << LOG2
    m = n // SHARDS
    return O.msm_canon(scalars(n)[k * m:(k + 1) * m], O.base_points(n, 5)[k * m:(k + 1) * m])


def _pippenger(c):
    from oracle import pyoracle
    O = pyoracle.Oracle()
    n = 1 << LOG2
    return O.msm_pippenger(scalars(n), O.base_points(n, 5), c)


def main():
    from oracle import pyoracle
    pyoracle.build()
    O, R = pyoracle.Oracle(), pyoracle.Reference()
    with mp.Pool(SHARDS) as pool:
        pip = pool.apply_async(_pippenger, (12,))   # the labelled alternative (orc_msm_pippenger, c = 12)
        roots = pool.map(_shard, range(SHARDS))
        oroots = pool.map(_shard_oracle, range(SHARDS))
        pip = pip.get()
    roots = np.stack(roots)
    res = R.point_tree(roots)
    assert np.array_equal(np.stack(oroots), roots) and np.array_equal(O.point_tree(roots), res), \
        "the CPU restatement disagrees with the reference build"
    d8 = lambda a: hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()[:16]
    out = {"n": 1 << LOG2, "source": "reference build (oracle/_ref/libbpref.so: ref_msm_canon per shard + "
                                     "ref_point_tree); the CPU restatement agrees",
           "points": "base_points(seed {5})", "scalars": "SHA256('msm-s'||i_le32), byte31&=0x7F",
           "digest": d8(res), "result": [int(x) for x in res],
           "shard_log2": LOG2 - 3, "shard_roots": [[int(x) for x in r] for r in roots],
           "pippenger_w12": {"digest": d8(pip), "result": [int(x) for x in pip]}}
    with open(os.path.join(HERE, "msm_2p20.json"), "w") as f:
        json.dump(out, f, indent=1)
    print("digest", out["digest"])


if __name__ == "__main__":
    main()
