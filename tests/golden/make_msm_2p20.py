"""Golden digest of the full-size configs[2] MSM (2^20 points), from the CPU restatement.

Inputs exactly as SURVEY §8(d) config 3 / §8c: points = generate_deterministic_base_points
with seed {5} (complete_bulletproof_test.cu:33-63: SHA-256 derived X, Y, Z = 1, T = X*Y),
scalars_i = SHA256("msm-s" || i_le32) with byte 31 &= 0x7F.  Result = the canonical-tree MSM
(cuda_bulletproof_kernels.cu:26-207 as point_multi_scalar_mul_shared_kernel defines it).

The canonical tree decomposes exactly over aligned power-of-two shards, so the
2^20 scalar multiplications run as 8 shards of 2^17 in 8 processes and the 8 shard roots are
combined by the oracle's point_tree: the same bits as one oracle.msm_canon over all points
(the 4096-point survey digest, test_msm_4096_survey_digest, pins that oracle to the reference).

    python tests/golden/make_msm_2p20.py      # ~1 min on 8 cores -> tests/golden/msm_2p20.json

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
    O = pyoracle.Oracle()
    n = 1 << LOG2
    m = n // SHARDS
    P = O.base_points(n, 5)[k * m:(k + 1) * m]
    s = scalars(n)[k * m:(k + 1) * m]
    return O.msm_canon(s, P)


def _pippenger(c):
    from oracle import pyoracle
    O = pyoracle.Oracle()
    n = 1 << LOG2
    return O.msm_pippenger(scalars(n), O.base_points(n, 5), c)


def main():
    from oracle import pyoracle
    O = pyoracle.Oracle()
    with mp.Pool(SHARDS + 1) as pool:
        pip = pool.apply_async(_pippenger, (12,))   # the labelled alternative (orc_msm_pippenger, c = 12)
        roots = pool.map(_shard, range(SHARDS))
        pip = pip.get()
    roots = np.stack(roots)
    res = O.point_tree(roots)
    d8 = lambda a: hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()[:16]
    out = {"n": 1 << LOG2, "points": "base_points(seed {5})", "scalars": "SHA256('msm-s'||i_le32), byte31&=0x7F",
           "digest": d8(res), "result": [int(x) for x in res],
           "shard_log2": LOG2 - 3, "shard_roots": [[int(x) for x in r] for r in roots],
           "pippenger_w12": {"digest": d8(pip), "result": [int(x) for x in pip]}}
    with open(os.path.join(HERE, "msm_2p20.json"), "w") as f:
        json.dump(out, f, indent=1)
    print("digest", out["digest"])


if __name__ == "__main__":
    main()
