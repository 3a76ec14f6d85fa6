"""Per-kernel totals from a rocprofv3 results database (rocpd sqlite), and optionally the timeline
of the last call that starts with a given kernel.
    python tools/prof_summary.py <results.db> [first_kernel_substring]"""
import sqlite3
import sys

c = sqlite3.connect(sys.argv[1])
rows = [(r[0].replace("(anonymous namespace)::", ""),) + tuple(r[1:]) for r in
        c.execute("select name, start, end, grid_x, stream_id, queue_id from kernels order by start")]
tot = {}
for r in rows:
    k = r[0].split("(")[0]
    n, t = tot.get(k, (0, 0))
    tot[k] = (n + 1, t + r[2] - r[1])
for k, (n, t) in sorted(tot.items(), key=lambda x: -x[1][1]):
    print(f"{k[-60:]:60s} {n:6d} {t / 1e6:9.3f} ms {t / n / 1e3:9.1f} us")
if len(sys.argv) > 2:
    idx = [i for i, r in enumerate(rows) if sys.argv[2] in r[0]]
    s0 = idx[-2] if len(idx) > 1 else idx[-1]
    t0 = rows[s0][1]
    for r in rows[s0:]:
        nm = r[0].split("(")[0].split("::")[-1][-36:]
        print(f"{nm:36s} q{r[5]} grid {r[3]:10d} start {(r[1] - t0) / 1e3:9.1f} dur {(r[2] - r[1]) / 1e3:8.1f} us")
