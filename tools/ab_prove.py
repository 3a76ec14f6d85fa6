"""A/B the prover between two builds of the library in one process each (tools/, not a test).

  python tools/ab_prove.py <lib.so> [B] [streams]
Times batch_generate_range_proof on random values, single stream and 2 streams alternating."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import cudabulletproof_amd as bp  # noqa: E402
from cudabulletproof_amd import synth  # noqa: E402

bp.LIB_PATH = os.path.abspath(sys.argv[1])
B = int(sys.argv[2]) if len(sys.argv) > 2 else 16384
n = 64
dev = torch.device("cuda:0")
G, H, g, h = synth.generators(n, dev)
T = lambda a: torch.from_numpy(np.ascontiguousarray(a).view(np.int64)).to(dev)
Gd, Hd, gd, hd = T(G), T(H), T(g), T(h)
pi = synth.prove_inputs(B, n)
args = [T(pi["v"]), T(pi["gamma"]), T(pi["sL"]), T(pi["sR"]), T(pi["rnd"])]
streams = [torch.cuda.Stream(dev) for _ in range(2)]
for ns in (1, 2):
    for st in streams[:ns]:
        with torch.cuda.stream(st):
            bp.batch_generate_range_proof(n, *args, Gd, Hd, gd, hd, stream=st)
    torch.cuda.synchronize()
    K = 6
    t0 = time.perf_counter()
    for k in range(K):
        st = streams[k % ns]
        with torch.cuda.stream(st):
            bp.batch_generate_range_proof(n, *args, Gd, Hd, gd, hd, stream=st)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / K
    print(f"{os.path.basename(sys.argv[1])} streams={ns} {dt * 1e3:7.2f} ms/batch {B / dt:9.0f} proofs/s", flush=True)
