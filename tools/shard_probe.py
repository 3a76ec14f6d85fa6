"""configs[4] rank-shard probe (one process, many schedules): one rank's shard of the 2^16-proof
batch (default 8192 proofs = N = 8) pushed through two verify pipelines on two streams, as
bench.py's sharded_2p16 leg does, timed for every (push batch, drain policy) pair.  The drain
policy is read per tick from the environment (HIPBP_QUAD, HIPBP_QUAD_MAX_ITEMS), so one process
A/Bs them; every run's verdict digest must be the same.

  python tools/shard_probe.py [shard] [push batches, comma-separated] [quad max items, comma-separated; 0 = off;
                                                                        "Q:P" also sets the pair bound P]
"""
import hashlib
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import cudabulletproof_amd as bp  # noqa: E402
from cudabulletproof_amd import synth  # noqa: E402

shard = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
# push schedules: "4096" = equal pushes of 4096; "4096+2048+1024+1024" = that sequence (must sum to the shard);
# pushes alternate over the two pipelines
def schedule(spec):
    if "+" in spec:
        seq = [int(x) for x in spec.split("+")]
        assert sum(seq) == shard, spec
        return seq
    b = int(spec)
    return [min(b, shard - j) for j in range(0, shard, b)]
pushes = [schedule(x) for x in (sys.argv[2] if len(sys.argv) > 2 else "1024,2048,4096").split(",")]
qmaxes = [x for x in (sys.argv[3] if len(sys.argv) > 3 else "0,49152,131072,262144").split(",")]
reps = int(os.environ.get("REPS", "3"))
RR = os.environ.get("RR", "0") == "1"   # round-robin drain after a sync on the pushes' first ticks
NP = int(os.environ.get("NP", "2"))   # pipelines (streams)
n, B = 64, 1024
dev = torch.device("cuda:0")
bp.lib()
G, H, g, h = synth.generators(n, dev)
T = lambda a: torch.from_numpy(np.ascontiguousarray(a).view(np.int64)).to(dev)
Gd, Hd, gd, hd = T(G), T(H), T(g), T(h)
gens = bp.Generators(n, Gd, Hd, gd, hd, prefix_bits=int(os.environ.get("K", "22")))
tiles = []
for t in range(4):
    pi = {k: T(v) for k, v in synth.prove_inputs(B, n, seed=5001 + t).items()}
    out = bp.batch_generate_range_proof(n, pi["v"], pi["gamma"], pi["sL"], pi["sR"], pi["rnd"], Gd, Hd, gd, hd,
                                        gens=gens)
    tiles.append({k: out[k] for k in bp.RangeProofBatch.FIELDS})
torch.cuda.synchronize()
# PRIO=1: the last pipeline's stream at high priority (its stage 0 starts behind the first's lane sort,
# so its drain ends last)
PRIO = os.environ.get("PRIO", "0") == "1"
streams = [torch.cuda.Stream(dev, priority=-1 if PRIO and i == NP - 1 else 0) for i in range(NP)]


def rows(j0, m):
    parts, j = [], j0
    while j < j0 + m:
        k = min(B - j % B, j0 + m - j)
        parts.append(((j // B) % 4, j % B, k))
        j += k
    return {f: torch.cat([tiles[t][f][r0:r0 + k] for t, r0, k in parts]) for f in bp.RangeProofBatch.FIELDS}


print(f"shard {shard} proofs, {NP} pipelines, K = {gens.bits}", flush=True)
for seq in pushes:
    Bs = max(seq)
    pipes = [bp.VerifyPipeline(Bs, n, Gd, Hd, hd, stream=streams[i]) for i in range(NP)]
    for pp in pipes:
        pp.use_gens(gens)
    jobs, j = [], 0
    for m in seq:
        jobs.append((j, m))
        j += m
    batches = [bp.RangeProofBatch(n, **rows(j0, m)) for j0, m in jobs]
    offs = np.cumsum([0] + [m for _, m in jobs])
    for qspec in qmaxes:
        qm = int(qspec.split(":")[0])
        os.environ["HIPBP_QUAD_MAX_ITEMS"] = str(qm)
        if ":" in qspec:
            os.environ["HIPBP_PAIR_MAX_ITEMS"] = qspec.split(":")[1]
        else:
            os.environ.pop("HIPBP_PAIR_MAX_ITEMS", None)
        if qm == 0:
            os.environ["HIPBP_QUAD"] = "0"
        else:
            os.environ.pop("HIPBP_QUAD", None)
        best, dig = None, None
        for r in range(reps + 1):
            ok = torch.zeros(shard, dtype=torch.uint8, device=dev)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for k, b in enumerate(batches):
                pipes[k % NP].push(b, ok[offs[k]:offs[k + 1]])
            if RR:   # wait out the pushes' first ticks, then drain the pipelines tick by tick in turn
                torch.cuda.synchronize()
                for _ in range(max(pp.depth for pp in pipes)):
                    for pp in pipes:
                        pp.push(None)
            for pp in pipes:
                pp.flush()
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            if r:
                best = dt if best is None else min(best, dt)
            d = hashlib.sha256(ok.cpu().numpy().tobytes()).hexdigest()[:16]
            assert dig is None or d == dig, (d, dig)
            dig = d
        print(f"push {'+'.join(map(str, seq)):24s}  quad:pair {qspec:>13s}  {best * 1e3:7.2f} ms  {shard / best / 1e3:7.1f} K verifies/s  "
              f"digest {dig}", flush=True)
    for pp in pipes:
        pp.close()
os.environ.pop("HIPBP_QUAD", None)
os.environ.pop("HIPBP_QUAD_MAX_ITEMS", None)
os.environ.pop("HIPBP_PAIR_MAX_ITEMS", None)
