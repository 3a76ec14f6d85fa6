"""Summarize a tools/profile_pip.sh run (gpurun_out/prof_<tag>_pip/) into profiles/.

    python tools/pip_prof_summary.py <tag>
      -> profiles/rocprof_<tag>_pip_summary.md   per-kernel totals and per-MSM times
      -> profiles/raw_<tag>_pip/kernel_stats.csv  rocprofv3's own --stats table
"""
import csv
import os
import shutil
import sys

tag = sys.argv[1]
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
src = os.path.join(root, "gpurun_out", f"prof_{tag}_pip")
rows = list(csv.DictReader(open(os.path.join(src, "trace", "run_kernel_trace.csv"))))
probe = open(os.path.join(src, "probe.txt")).read().strip()
tot = {}
for r in rows:
    k = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0]
    if "rocprim" in k:
        k = "rocprim " + ("histogram" if "histogram" in r["Kernel_Name"] else
                          "onesweep" if "onesweep" in r["Kernel_Name"] else
                          "scan/lookback" if ("lookback" in r["Kernel_Name"] or "scan" in r["Kernel_Name"]) else "other")
    n, t = tot.get(k, (0, 0))
    tot[k] = (n + 1, t + int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
nmsm = sum(n for k, (n, _) in tot.items() if k.endswith("k_pip_horner")) // 2
all_ns = sum(t for _, t in tot.values())
out = [f"# rocprofv3 summary — {tag}, Pippenger MSM alone", "",
       f"Command: `tools/profile_pip.sh {tag}` on one MI355X: `rocprofv3 --kernel-trace --stats -- python3 "
       "tools/pip_probe.py 20 12 12 2` (2^20 config-3 points, window 12: one warm-up + 12 single-stream MSMs, then one "
       "warm-up per stream + 12 MSMs alternating over two streams, each checked equal). "
       f"{nmsm} MSMs under the profiler (k_pip_horner: 2 launches per MSM). Probe output (under the profiler, which "
       "serialises part of the two-stream overlap):", "", "```", probe, "```", "",
       "| kernel | calls | total ms | avg ms | per MSM ms | % GPU time |", "|---|---|---|---|---|---|"]
for k, (n, t) in sorted(tot.items(), key=lambda x: -x[1][1]):
    out.append(f"| {k} | {n} | {t / 1e6:.3f} | {t / n / 1e6:.4f} | {t / nmsm / 1e6:.4f} | {100 * t / all_ns:.1f} |")
out.append(f"| **all kernels** |  | {all_ns / 1e6:.3f} |  | {all_ns / nmsm / 1e6:.3f} | 100 |")
out += ["", "Per MSM, the kernel time adds to more than the wall time of one call because the top part's chunks, "
        "window trees and Horner run on the side stream beside the bottom part's bucket trees (DESIGN §9, profiles/NOTES.md §7c)."]
# PMC passes (profile_pip.sh): per kernel, summed over its launches in the 3-MSM probe runs,
# per MSM; HBM bytes = 2 x FETCH_SIZE + WRITE_SIZE (KB; gfx950 FETCH_SIZE x2 correction)
def counters(name):
    path = os.path.join(src, f"pmc_{name}", "run_counter_collection.csv")
    if not os.path.exists(path):
        return None
    per = {}
    for r in csv.DictReader(open(path)):
        d = per.setdefault(int(r["Dispatch_Id"]), {"kernel": r["Kernel_Name"].replace("(anonymous namespace)::", "")
                                                      .split("(")[0],
                                                   "dur": int(r["End_Timestamp"]) - int(r["Start_Timestamp"])})
        d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return per


pm = {k: counters(k) for k in ("fetch", "write", "valu", "cyc", "busy", "tcc")}
if pm["fetch"]:
    nm = 4   # pip_probe.py 20 12 3 1: one warm-up + 3 timed MSMs
    kern = sorted({d["kernel"] for d in pm["fetch"].values() if d["kernel"].startswith("bp::k_pip")})

    def agg(name, key, k, f=sum):
        ds = [d.get(key, 0.0) for d in (pm[name] or {}).values() if d["kernel"] == k]
        return f(ds) if ds else float("nan")

    def avg(xs):
        return sum(xs) / len(xs)
    out += ["", "## PMC counters per MSM (`rocprofv3 --pmc`, one pass per counter group, 4 MSMs on one stream)", "",
            "| kernel | launches/MSM | ms/MSM | HBM MB/MSM (2xFETCH+WRITE) | GB/s | VALU winstr/MSM (M) | VALUBusy % "
            "| VALUUtil % | L2 hit % | eff. clock GHz |", "|---|---|---|---|---|---|---|---|---|---|"]
    for k in kern:
        n = sum(1 for d in pm["fetch"].values() if d["kernel"] == k) / nm
        dur = agg("fetch", "dur", k) / nm / 1e6
        hbm = (2 * agg("fetch", "FETCH_SIZE", k) + agg("write", "WRITE_SIZE", k)) * 1024 / nm
        vi = agg("valu", "SQ_INSTS_VALU", k) / nm
        bd = [(d.get("VALUBusy", 0.0), d.get("VALUUtilization", 0.0), d["dur"]) for d in (pm["busy"] or {}).values()
              if d["kernel"] == k]
        tw = sum(x[2] for x in bd) or 1
        busy = sum(x[0] * x[2] for x in bd) / tw   # duration-weighted over the launches
        util = sum(x[1] * x[2] for x in bd) / tw
        hit, miss = agg("tcc", "TCC_HIT_sum", k), agg("tcc", "TCC_MISS_sum", k)
        grbm = agg("cyc", "GRBM_GUI_ACTIVE", k)
        cdur = agg("cyc", "dur", k)
        out.append(f"| {k.replace('bp::', '')} | {n:.1f} | {dur:.3f} | {hbm / 1e6:.1f} | {hbm / (dur * 1e-3) / 1e9:.0f} | "
                   f"{vi / 1e6:.1f} | {busy:.1f} | {util:.1f} | {100 * hit / max(hit + miss, 1):.1f} | "
                   f"{grbm / 8 / cdur:.2f} |")
    out += ["", "Algorithmic bytes per MSM (SURVEY §8(d)): 2^20 x (128 B point + 32 B scalar) + 128 B = 167.8 MB. "
            "GB/s is per kernel over its own launch time under the profiler (serialised). VALUBusy and VALUUtil "
            "are weighted by launch duration. The clock column (GRBM_GUI_ACTIVE / 8 / duration) is meaningful "
            "only for kernels that run for a good fraction of a millisecond."]
dst = os.path.join(root, "profiles", f"rocprof_{tag}_pip_summary.md")
open(dst, "w").write("\n".join(out) + "\n")
os.makedirs(os.path.join(root, "profiles", f"raw_{tag}_pip"), exist_ok=True)
shutil.copy(os.path.join(src, "trace", "run_kernel_stats.csv"),
            os.path.join(root, "profiles", f"raw_{tag}_pip", "kernel_stats.csv"))
print(dst)
