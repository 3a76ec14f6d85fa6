"""Prover throughput vs number of streams / priorities (tools/, not a test).

  python tools/ab_streams.py [B]"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import cudabulletproof_amd as bp  # noqa: E402
from cudabulletproof_amd import synth  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
n = 64
dev = torch.device("cuda:0")
print("priority range", torch.cuda.Stream.priority_range(), flush=True)
G, H, g, h = synth.generators(n, dev)
T = lambda a: torch.from_numpy(np.ascontiguousarray(a).view(np.int64)).to(dev)
Gd, Hd, gd, hd = T(G), T(H), T(g), T(h)
pi = synth.prove_inputs(B, n)
args = [T(pi["v"]), T(pi["gamma"]), T(pi["sL"]), T(pi["sR"]), T(pi["rnd"])]
for prios in ((0, -1), (0, -1, 0, -1)):
    streams = [torch.cuda.Stream(dev, priority=p) for p in prios]
    outs = [None] * len(streams)
    for i, st in enumerate(streams):
        outs[i] = bp.batch_generate_range_proof(n, *args, Gd, Hd, gd, hd, stream=st)
    torch.cuda.synchronize()
    K = 8
    t0 = time.perf_counter()
    for k in range(K):
        outs[k % len(streams)] = bp.batch_generate_range_proof(n, *args, Gd, Hd, gd, hd, stream=streams[k % len(streams)])
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / K
    print(f"prios={prios} {dt * 1e3:7.2f} ms/batch {B / dt:9.0f} proofs/s", flush=True)
