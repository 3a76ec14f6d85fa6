"""Run hipbp_msm_pippenger on the 2^20 config-3 inputs a few times (for rocprofv3).
    python tools/pip_probe.py [log2_n] [window_bits] [reps]"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import cudabulletproof_amd as bp  # noqa: E402
from cudabulletproof_amd import synth  # noqa: E402

lg = int(sys.argv[1]) if len(sys.argv) > 1 else 20
c = int(sys.argv[2]) if len(sys.argv) > 2 else 12
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
dev = torch.device("cuda:0")
bp.lib()
s, P = synth.msm_config3(0, 1 << lg, dev)
T = lambda a: torch.from_numpy(np.ascontiguousarray(a).view(np.int64)).to(dev)
sd, Pd = T(s), T(P)
out = torch.zeros(16, dtype=torch.int64, device=dev)
bp.msm_pippenger(out, sd, Pd, c)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(reps):
    bp.msm_pippenger(out, sd, Pd, c)
torch.cuda.synchronize()
print(f"n=2^{lg} c={c}: {(time.perf_counter() - t0) / reps * 1e3:.3f} ms")
