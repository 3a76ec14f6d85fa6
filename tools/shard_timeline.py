"""Timeline of the last shard run in a tools/shard_trace_bench.sh kernel trace: every kernel of the last
run (the launches after the last gap of > 3 ms with nothing running), per queue, relative to the run's
first launch; then the time the GPU ran nothing but latency-bound (small-grid) ticks.

  python tools/shard_timeline.py <tag>
"""
import csv
import glob
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
tag = sys.argv[1] if len(sys.argv) > 1 else "r03n"
path = glob.glob(os.path.join(ROOT, "gpurun_out", f"shard_trace_{tag}", "**", "*kernel_trace.csv"), recursive=True)[0]
rows = list(csv.DictReader(open(path)))


def short(n):
    n = n.replace("(anonymous namespace)::", "").split("(")[0].replace("bp::", "")
    n = n[5:] if n.startswith("void ") else n
    return n[:40]


ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]), int(r["Grid_Size_X"]),
             r.get("Queue_Id", r.get("Stream_Id", "?"))) for r in rows)
# split into runs at idle gaps
start = 0
busy_until = ev[0][1]
for i in range(1, len(ev)):
    if ev[i][0] - busy_until > 3_000_000:
        start = i
    busy_until = max(busy_until, ev[i][1])
run = ev[start:]
t0 = run[0][0]
t1 = max(e[1] for e in run)
print(f"last run: {len(run)} kernels, {(t1 - t0) / 1e6:.2f} ms")
for s, e, k, g, q in run:
    if (e - s) > 50_000 or k.startswith("k_terms"):
        print(f"q{q:>3} {(s - t0) / 1e6:8.3f} {(e - t0) / 1e6:8.3f} {(e - s) / 1e6:7.3f}  {k:40s} grid {g}")
