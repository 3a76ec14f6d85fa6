"""Table-driven A/B runner for bench.py on the GPU box (tools/, not a test).

Every configuration is a name plus tokens: `env:KEY=VALUE` (environment), `lib:PATH` (a prebuilt
library swapped in as the product library for that run; the original is restored at the end) or
plain bench.py arguments.  Configurations run alternately, `--reps` times each, one bench.py child
process per run under its own time limit; the first failing run ends the A/B (no retries).

  python tools/ab.py --tag r05k --reps 2 --base "--no-cpu --no-ipa --no-msm --no-shard --no-host" \
      --cfg "K16: --prefix-bits 16" --cfg "K23: --prefix-bits 23" \
      --pick value --pick repeats.median --pick prove.value

  (replaces the round 1-4 scripts ab_env / ab_libs / ab_pipes / ab_prefix_bits / ab_prove_gate /
   ab_run / ab_shard_env / ab_prove / ab_streams: e.g. a library A/B is --cfg "base: lib:ab/lib_base.so"
   --cfg "occ3: lib:ab/lib_occ3.so", an environment A/B --cfg "gate: env:HIPBP_PROVE_GATE=1")

Writes gpurun_out/ab/<tag>_<name>_r<rep>.json (the bench line) and gpurun_out/ab/<tag>.json
(every run's picked fields + per-configuration medians) and prints one row per run.
"""
import argparse
import json
import os
import shlex
import shutil
import statistics
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "cudabulletproof_amd", "libcudabulletproof_hip.so")


def pick(d, path):
    for k in path.split("."):
        if not isinstance(d, dict) or k not in d:
            return None
        d = d[k]
    return d


def parse_cfg(spec):
    name, _, rest = spec.partition(":")
    env, lib, args = {}, None, []
    for tok in shlex.split(rest):
        if tok.startswith("env:"):
            k, _, v = tok[4:].partition("=")
            env[k] = v
        elif tok.startswith("lib:"):
            lib = tok[4:]
        else:
            args.append(tok)
    return {"name": name.strip(), "env": env, "lib": lib, "args": args}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tag", required=True)
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--base", default="", help="bench.py arguments common to every configuration")
    ap.add_argument("--cfg", action="append", required=True, help='"name: tokens" (see the module docstring)')
    ap.add_argument("--pick", action="append", default=None, help="dotted JSON fields to tabulate (default: value)")
    ap.add_argument("--timeout", type=int, default=400, help="seconds per bench.py run")
    a = ap.parse_args()
    cfgs = [parse_cfg(c) for c in a.cfg]
    fields = a.pick or ["value"]
    out_dir = os.path.join(ROOT, "gpurun_out", "ab")
    os.makedirs(out_dir, exist_ok=True)
    saved = None
    if any(c["lib"] for c in cfgs):
        saved = LIB + ".ab_saved"
        shutil.copy2(LIB, saved)
    rows = []
    try:
        for rep in range(1, a.reps + 1):
            for c in cfgs:
                if c["lib"]:
                    shutil.copy2(os.path.join(ROOT, c["lib"]), LIB)
                elif saved:
                    shutil.copy2(saved, LIB)
                cmd = ["timeout", "-k", "10", str(a.timeout), sys.executable, "-u", os.path.join(ROOT, "bench.py")]
                cmd += shlex.split(a.base) + c["args"]
                path = os.path.join(out_dir, f"{a.tag}_{c['name']}_r{rep}.json")
                with open(path, "w") as fo, open(path[:-5] + ".err", "w") as fe:
                    rc = subprocess.call(cmd, stdout=fo, stderr=fe, cwd=ROOT, env=dict(os.environ, **c["env"]))
                if rc != 0:
                    print(f"{c['name']} rep {rep}: bench.py exited {rc} (see {path[:-5]}.err); A/B stopped", flush=True)
                    sys.exit(1)
                line = json.loads(open(path).read().strip().splitlines()[-1])
                row = {"cfg": c["name"], "rep": rep, **{f: pick(line, f) for f in fields}}
                rows.append(row)
                print(json.dumps(row), flush=True)
    finally:
        if saved:
            shutil.move(saved, LIB)
    summary = {}
    for c in cfgs:
        mine = [r for r in rows if r["cfg"] == c["name"]]
        summary[c["name"]] = {f: statistics.median([r[f] for r in mine if isinstance(r[f], (int, float))])
                              if any(isinstance(r[f], (int, float)) for r in mine) else None for f in fields}
        summary[c["name"]]["spec"] = {k: c[k] for k in ("env", "lib", "args")}
    json.dump({"tag": a.tag, "base": a.base, "reps": a.reps, "runs": rows, "median": summary},
              open(os.path.join(out_dir, f"{a.tag}.json"), "w"), indent=1)
    for name, s in summary.items():
        print(name, {f: (round(v) if isinstance(v, float) and v > 100 else v) for f, v in s.items() if f != "spec"})


if __name__ == "__main__":
    main()
