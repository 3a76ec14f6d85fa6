"""Smoke each named batch field op (bp.field_op) on 1024 random elements, one line per op, stopping at the
first failure (tools/, not a test): python tools/field_op_probe.py add sub mul ..."""
import sys, os
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
import numpy as np, torch
import cudabulletproof_amd as bp
dev = torch.device("cuda:0")
rng = np.random.default_rng(1)
a = torch.from_numpy(rng.integers(0, 2**63, (1024, 4), dtype=np.int64)).to(dev)
b = torch.from_numpy(rng.integers(0, 2**63, (1024, 4), dtype=np.int64)).to(dev)
for op in sys.argv[1:]:
    r = torch.empty_like(a)
    try:
        bp.field_op(op, r, a, b); torch.cuda.synchronize(); print(op, "ok", flush=True)
    except Exception as e:
        print(op, "FAIL", e, flush=True); break
