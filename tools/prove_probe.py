"""Time the GPU prover on value patterns that change its work mix (tools/, not a test).

  python tools/prove_probe.py [B]
all-ones values: aR = 0 everywhere (only sL/sR/gamma/alpha/rho are full scalar-mults);
zero values: every aR_i = sub(0, 1), a 255-bit scalar with popcount 251; random: half each."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import cudabulletproof_amd as bp  # noqa: E402
from cudabulletproof_amd import synth  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
n = 64
dev = torch.device("cuda:0")
G, H, g, h = synth.generators(n, dev)
T = lambda a: torch.from_numpy(np.ascontiguousarray(a).view(np.int64)).to(dev)
Gd, Hd, gd, hd = T(G), T(H), T(g), T(h)
pi = synth.prove_inputs(B, n)
PATTERNS = (("random", None), ("ones", np.uint64(2**64 - 1)), ("zero", np.uint64(0)))
sel = sys.argv[2:] or [p[0] for p in PATTERNS]
for name, fill in [p for p in PATTERNS if p[0] in sel]:
    v = pi["v"].copy()
    if fill is not None:
        v[:, 0] = fill
    args = [T(v), T(pi["gamma"]), T(pi["sL"]), T(pi["sR"]), T(pi["rnd"])]
    bp.batch_generate_range_proof(n, *args, Gd, Hd, gd, hd)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    out = bp.batch_generate_range_proof(n, *args, Gd, Hd, gd, hd)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    print(f"{name:7s} B={B} {dt * 1e3:8.2f} ms  {B / dt:9.0f} proofs/s  valid={int(out['valid'].sum())}", flush=True)
