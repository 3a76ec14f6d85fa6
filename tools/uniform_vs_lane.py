"""Time per scalar-mult: wave-uniform scalars (sm_uniform: squarings, Z2 = 1 add) vs per-lane
scalars (the unified step), 2^20-point hipbp_msm, same chain length (255 bits, popcount 128)."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import cudabulletproof_amd as bp  # noqa: E402
from cudabulletproof_amd import synth  # noqa: E402

n = 1 << 20
dev = torch.device("cuda:0")
bp.lib()
_, pts = synth.msm_inputs(n)
rng = np.random.default_rng(1)


def scalar_with(pop):
    bits = np.zeros(256, np.uint8)
    bits[254] = 1
    idx = rng.choice(254, pop - 1, replace=False)
    bits[idx] = 1
    v = np.packbits(bits, bitorder="little").view("<u8").astype(np.uint64)
    return v


lane = np.stack([scalar_with(128) for _ in range(4096)])
lane = np.tile(lane, (n // 4096, 1))
uni = np.tile(scalar_with(128), (n, 1))
T = lambda a: torch.from_numpy(np.ascontiguousarray(a).view(np.int64)).to(dev)
Pd = T(pts)
out = torch.zeros(16, dtype=torch.int64, device=dev)
for name, sc in (("per-lane", lane), ("uniform", uni)):
    sd = T(sc)
    bp.msm(out, sd, Pd)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(3):
        bp.msm(out, sd, Pd)
    torch.cuda.synchronize()
    print(f"{name}: {(time.perf_counter() - t0) / 3 * 1e3:.3f} ms per 2^20 scalar-mults", flush=True)
