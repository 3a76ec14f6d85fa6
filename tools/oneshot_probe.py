"""Per-call latency of the drop-in entry point cuda_range_proof_verify (one proof per call, warm),
through the reference's own benchmark hook cuda_benchmark_range_proof (tools/, not a test).

  python tools/oneshot_probe.py [iterations] [bit sizes, comma-separated]
"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import cudabulletproof_amd as bp  # noqa: E402

it = int(sys.argv[1]) if len(sys.argv) > 1 else 20
sizes = [int(x) for x in (sys.argv[2] if len(sys.argv) > 2 else "16,64").split(",")]
L = bp.lib()
for n in sizes:
    L.cuda_benchmark_range_proof(ctypes.c_int(it), ctypes.c_size_t(n))
