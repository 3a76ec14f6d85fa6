"""Run hipbp_msm_pippenger on the 2^20 config-3 inputs (for rocprofv3 and stream / batch A/B runs).
    python tools/pip_probe.py [log2_n] [window_bits] [reps] [streams] [batch]
streams > 1: reps MSMs rotate over that many streams (independent workspaces); prints the
throughput and checks every result against the single-stream one.  batch > 1: batches of that
many MSMs over the same points (hipbp_msm_pippenger_batch; MSM m's scalars are the config-3
scalars rolled by m rows), each result checked against a single call."""
import hashlib
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
ns = int(sys.argv[4]) if len(sys.argv) > 4 else 1
nbat = int(sys.argv[5]) if len(sys.argv) > 5 else 1
dev = torch.device("cuda:0")
bp.lib()
s, P = synth.msm_config3(0, 1 << lg, dev)
T = lambda a: torch.from_numpy(np.ascontiguousarray(a).view(np.int64)).to(dev)
sd, Pd = T(s), T(P)
out = torch.zeros(16, dtype=torch.int64, device=dev)
bp.msm_pippenger(out, sd, Pd, c)
torch.cuda.synchronize()
ref = hashlib.sha256(out.cpu().numpy().tobytes()).hexdigest()[:16]
t0 = time.perf_counter()
for _ in range(reps):
    bp.msm_pippenger(out, sd, Pd, c)
torch.cuda.synchronize()
dt = (time.perf_counter() - t0) / reps
print(f"n=2^{lg} c={c}: {dt * 1e3:.3f} ms  {(1 << lg) / dt / 1e6:.1f} M points/s  digest {ref}", flush=True)
if nbat > 1:
    sb = torch.cat([torch.roll(sd, m, 0) for m in range(nbat)]).contiguous()
    want = torch.zeros(nbat, 16, dtype=torch.int64, device=dev)
    for m in range(nbat):
        bp.msm_pippenger(want[m], sb[m << lg:(m + 1) << lg], Pd, c)
    # outs below are zero-filled on torch's default stream; without this sync the fill can run
    # after a batch issued on a (non-blocking) side stream has written its results
    torch.cuda.synchronize()
    want_s = torch.zeros(nbat, 16, dtype=torch.int64, device=dev)
    for m in range(nbat):
        bp.msm_pippenger(want_s[m], sb[m << lg:(m + 1) << lg], Pd, c)
        torch.cuda.synchronize()
    w_ok = bool((want == want_s).all().item())
    st = [torch.cuda.Stream(dev) for _ in range(max(ns, 1))]
    outs = [torch.zeros(nbat, 16, dtype=torch.int64, device=dev) for _ in range(max(ns, 1))]
    for i in range(len(st)):
        bp.msm_pippenger_batch(outs[i], sb, Pd, c, stream=st[i])
    torch.cuda.synchronize()
    ok = all(bool((o == want).all().item()) for o in outs)
    ok1 = ok
    t0 = time.perf_counter()
    for k in range(reps):
        bp.msm_pippenger_batch(outs[k % len(st)], sb, Pd, c, stream=st[k % len(st)])
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / reps / nbat
    ok = ok and all(bool((o == want).all().item()) for o in outs)
    print(f"  batch {nbat} x {len(st)} streams: {dt * 1e3:.3f} ms per MSM  {(1 << lg) / dt / 1e6:.1f} M points/s  "
          f"same bits: {ok} (singles stable {w_ok}, first batch {ok1})", flush=True)
elif ns > 1:
    st = [torch.cuda.Stream(dev) for _ in range(ns)]
    outs = [torch.zeros(reps, 16, dtype=torch.int64, device=dev) for _ in range(ns)]
    for i in range(ns):   # warm each stream's workspace
        bp.msm_pippenger(outs[i][0], sd, Pd, c, stream=st[i])
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(reps):
        bp.msm_pippenger(outs[k % ns][k], sd, Pd, c, stream=st[k % ns])
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / reps
    ok = all(hashlib.sha256(outs[k % ns][k].cpu().numpy().tobytes()).hexdigest()[:16] == ref for k in range(reps))
    print(f"  {ns} streams: {dt * 1e3:.3f} ms per MSM  {(1 << lg) / dt / 1e6:.1f} M points/s  same bits: {ok}",
          flush=True)
