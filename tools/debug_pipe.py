import sys, os, numpy as np, torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import cudabulletproof_amd as bp
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
from test_gpu_parity import _batch_from_golden, _proof
n = int(sys.argv[1]) if len(sys.argv) > 1 else 16
d = dict(np.load(f"tests/golden/proofs_n{n}.npz"))
arrays = _batch_from_golden(bp, d, None)
dev = torch.device("cuda:0")
T = lambda a: torch.from_numpy(np.ascontiguousarray(a, np.uint64).view(np.int64)).to(dev)
print("single:", [bp.cuda_range_proof_verify(_proof(d, i), d["V"][i], n, d["G"], d["H"], d["g"], d["h"]) for i in range(6)])
print("single again:", [bp.cuda_range_proof_verify(_proof(d, i), d["V"][i], n, d["G"], d["H"], d["g"], d["h"]) for i in range(6)])
print("want:", d["ok_cuda"].tolist())
pipe = bp.VerifyPipeline(8, n, T(d["G"]), T(d["H"]), T(d["h"]))
for i in range(6):
    sub = {k: v[i:i+1] for k, v in arrays.items()}
    b = bp.RangeProofBatch.from_numpy(n, sub, dev)
    ok = torch.zeros(1, dtype=torch.uint8, device=dev); P = torch.zeros(1, 16, dtype=torch.int64, device=dev); c = torch.zeros(1, 16, dtype=torch.int64, device=dev)
    pipe.push(b, ok, P, c); pipe.flush(); torch.cuda.synchronize()
    print(i, ok.item(), np.array_equal(P.cpu().numpy().view(np.uint64)[0], d["P"][i]), np.array_equal(c.cpu().numpy().view(np.uint64)[0], d["check"][i]))
