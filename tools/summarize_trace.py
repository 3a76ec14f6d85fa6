"""Per-kernel summary of a rocprofv3 --kernel-trace CSV (any command), as a markdown table.

    python tools/summarize_trace.py <run_kernel_trace.csv> <title> [out.md]
"""
import collections
import csv
import re
import sys


def main():
    path, title = sys.argv[1], sys.argv[2]
    rows = list(csv.DictReader(open(path)))
    agg = collections.defaultdict(lambda: [0, 0.0, 1e30, 0.0])
    for r in rows:
        n = r["Kernel_Name"]
        m = re.search(r"bp::(?:\(anonymous namespace\)::)?(k_\w+)", n)
        n = m.group(1) if m else n.split("(")[0][:90]
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
        a = agg[n]
        a[0] += 1
        a[1] += d
        a[2] = min(a[2], d)
        a[3] = max(a[3], d)
    tot = sum(v[1] for v in agg.values())
    out = [f"# {title}", "", "| kernel | calls | total ms | avg ms | min ms | max ms | % time |",
           "|---|---|---|---|---|---|---|"]
    for k, v in sorted(agg.items(), key=lambda x: -x[1][1]):
        out.append(f"| {k} | {v[0]} | {v[1]:.3f} | {v[1] / v[0]:.3f} | {v[2]:.3f} | {v[3]:.3f} | {100 * v[1] / tot:.1f} |")
    text = "\n".join(out) + "\n"
    if len(sys.argv) > 3:
        open(sys.argv[3], "w").write(text)
    print(text)


if __name__ == "__main__":
    main()
