"""Predict the window-sharded Pippenger's per-MSM time at N ranks on one GPU: for each emulated
rank, the time of its window range (hipbp_msm_pippenger_windows), then the Horner alone.
  python tools/pip_shard_probe.py [log2 n] [window_bits]"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import cudabulletproof_amd as bp  # noqa: E402
from cudabulletproof_amd import shard, synth  # noqa: E402


def timed(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / reps * 1e3


def main():
    k = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    c = int(sys.argv[2]) if len(sys.argv) > 2 else 12
    dev = torch.device("cuda:0")
    n = 1 << k
    sc, pts = synth.msm_config3(0, n, dev)
    sd = torch.from_numpy(sc.view("int64")).to(dev)
    pd = pts if torch.is_tensor(pts) else torch.from_numpy(pts.view("int64")).to(dev)
    W = bp.pippenger_num_windows(c)
    out = torch.zeros(16, dtype=torch.int64, device=dev)
    Sw = torch.zeros(W, 16, dtype=torch.int64, device=dev)
    print(f"n=2^{k} c={c}: msm_pippenger {timed(lambda: bp.msm_pippenger(out, sd, pd, c)):.3f} ms")
    print(f"  horner alone {timed(lambda: bp.msm_pippenger_horner(out, Sw, c)):.3f} ms")
    for world in (1, 2, 4, 8):
        per = []
        for r in range(world):
            w0, w1 = shard.pippenger_window_bounds(c, world, r)
            per.append(timed(lambda: bp.msm_pippenger_windows(Sw, sd, pd, w0, w1, c)))
        print(f"  N={world}: window ranges ms " + " ".join(f"{x:.3f}" for x in per) + f"  max {max(per):.3f}")


if __name__ == "__main__":
    main()
