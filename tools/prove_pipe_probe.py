"""The bench's prove leg on its own (tools/, not a test): B proofs per batch (default 65536), the
generator set's K-bit prefix tables (default 22), batches alternating over S streams of different
priorities, `steps` timed batches — for rocprofv3 kernel traces of the prover's overlap.

  python tools/prove_pipe_probe.py [B] [streams] [steps] [K]
"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import cudabulletproof_amd as bp  # noqa: E402
from cudabulletproof_amd import synth  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
ns = int(sys.argv[2]) if len(sys.argv) > 2 else 2
steps = int(sys.argv[3]) if len(sys.argv) > 3 else 4
K = int(sys.argv[4]) if len(sys.argv) > 4 else 22
n = 64
dev = torch.device("cuda:0")
G, H, g, h = synth.generators(n, dev)
T = lambda a: torch.from_numpy(np.ascontiguousarray(a).view(np.int64)).to(dev)
Gd, Hd, gd, hd = T(G), T(H), T(g), T(h)
gens = bp.Generators(n, Gd, Hd, gd, hd, prefix_bits=K) if K else None
pi = {k: T(v) for k, v in synth.prove_inputs(B, n).items()}
lo, hi = torch.cuda.Stream.priority_range()
streams = [torch.cuda.Stream(dev, priority=max(hi, lo - k)) for k in range(ns)]
torch.cuda.synchronize()
run = lambda k: bp.batch_generate_range_proof(n, pi["v"], pi["gamma"], pi["sL"], pi["sR"], pi["rnd"], Gd, Hd, gd, hd,
                                              stream=streams[k % ns], gens=gens)
outs = [run(k) for k in range(ns)]
torch.cuda.synchronize()
t0 = time.perf_counter()
for k in range(steps):
    outs[k % ns] = run(k)
torch.cuda.synchronize()
dt = (time.perf_counter() - t0) / steps
same = all(torch.equal(outs[0][k], outs[-1][k]) for k in ("A", "S", "T1", "L", "R"))
print(f"B={B} streams={ns} K={K}: {dt * 1e3:.2f} ms per batch  {B / dt / 1e3:.1f} K proofs/s  same={same}", flush=True)
