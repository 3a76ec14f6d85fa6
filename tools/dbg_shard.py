import sys, numpy as np, torch
sys.path.insert(0, '.')
import cudabulletproof_amd as bp
from cudabulletproof_amd import synth
dev = torch.device('cuda:0')
n, B = 64, 1024
G, H, g, h = synth.generators(n, dev)
T = lambda a: torch.from_numpy(np.ascontiguousarray(a).view(np.int64)).to(dev)
Gd, Hd, gd, hd = T(G), T(H), T(g), T(h)
gens = bp.Generators(n, Gd, Hd, gd, hd, prefix_bits=16)
for seed in (1, 2, 5001, 5002):
    pi = {k: T(v) for k, v in synth.prove_inputs(B, n, seed=seed).items()}
    out = bp.batch_generate_range_proof(n, pi["v"], pi["gamma"], pi["sL"], pi["sR"], pi["rnd"], Gd, Hd, gd, hd, gens=gens)
    out0 = bp.batch_generate_range_proof(n, pi["v"], pi["gamma"], pi["sL"], pi["sR"], pi["rnd"], Gd, Hd, gd, hd)
    torch.cuda.synchronize()
    same = all(torch.equal(out[k], out0[k]) for k in bp.RangeProofBatch.FIELDS)
    b = bp.RangeProofBatch(n, **{k: out[k] for k in bp.RangeProofBatch.FIELDS})
    ok = torch.zeros(B, dtype=torch.uint8, device=dev)
    bp.batch_range_proof_verify(b, Gd, Hd, gd, hd, ok)
    torch.cuda.synchronize()
    print(seed, same, int(out["valid"].sum()), int(ok.sum()))
