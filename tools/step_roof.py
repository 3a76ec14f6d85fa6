"""Summarize the VALU microbenchmarks of one profiling call into profiles/valu_step_roof.json.

  python tools/step_roof.py <tag>     (reads gpurun_out/ubench_step_<tag>.json, ubench_step_pmc_<tag>/,
                                       ubench_issue_<tag>.json or the latest ubench_issue_*.json)

ubench_step: k_terms' point-operation loops (per-lane unified step, uniform doubling, uniform add)
from registers and LDS at k_terms' occupancy: VALU wave-instructions per second (SQ_INSTS_VALU
of the timed launch / its duration) and the shader clock during the loop (clock64 / wall_clock64).
ubench_issue: per-opcode issue cycles at 8 waves/SIMD in shader-clock cycles.
"""
import collections
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
tag = sys.argv[1]
g = lambda p: os.path.join(ROOT, "gpurun_out", p)
step = json.load(open(g(f"ubench_step_{tag}.json")))["kernels"]
per = collections.defaultdict(dict)
for r in csv.DictReader(open(g(f"ubench_step_pmc_{tag}/run_counter_collection.csv"))):
    k = int(r["Dispatch_Id"])
    per[k]["kernel"] = r["Kernel_Name"].split("(")[0].replace("void ", "")
    per[k]["dur"] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    per[k][r["Counter_Name"]] = per[k].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
names = {"k_step<0>": "step", "k_step<1>": "dbl", "k_step<2>": "add"}
out = {"tag": tag, "occupancy_waves_per_simd": 4, "kernels": {}}
for k, v in sorted(per.items()):
    nm = names.get(v["kernel"])
    if nm is None:
        continue
    rate = v["SQ_INSTS_VALU"] / (v["dur"] * 1e-9)   # the later (timed, warm) launch overwrites the first
    ghz = step[nm]["ghz"]
    out["kernels"][nm] = {"valu_per_wave": v["SQ_INSTS_VALU"] / v["SQ_WAVES"], "Ginstr_per_s": rate / 1e9,
                          "ghz": ghz, "cycles_per_instr_per_simd": 1024 * ghz * 1e9 / rate}
issue = sorted(glob.glob(g(f"ubench_issue_{tag}.json"))) or sorted(glob.glob(g("ubench_issue_*.json")))
if issue:
    out["issue_cycles_8waves"] = {k: v["cycles"] for k, v in json.load(open(issue[-1]))["ops"].items()}
    out["issue_source"] = os.path.basename(issue[-1])
json.dump(out, open(os.path.join(ROOT, "profiles", "valu_step_roof.json"), "w"), indent=1)
print(json.dumps(out, indent=1))
