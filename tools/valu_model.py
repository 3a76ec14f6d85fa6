"""VALU issue-cost model of the verify's hot loop -> profiles/valu_issue_model.json (read by bench.py).

  python tools/valu_model.py profiles/valu_issue_costs.json

Inputs: the per-opcode issue costs tools/ubench_issue.hip measured on the GPU (cycles per wave64
instruction per SIMD, in shader-clock cycles, 8 waves/SIMD, independent chains) and the opcode mix
of the point operations as compiled for gfx950 (tools/isa_ops.hip, common path, as
tools/isa_count.py counts it).  Output: the cycles one VALU instruction of that mix takes at full
issue (the instruction-weighted mean cost), per probe kernel; bench.py turns the one of the
per-lane unified step (the dominant loop of k_terms) into a peak: 1024 SIMDs x clock / cycles.
s_nop and other scalar instructions are not VALU issue and are left out (at 4 waves per SIMD the
SIMD issues another wave's VALU instruction in their slot).
"""
import collections
import json
import os
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
PROBES = ("p_ge_add_sel_zone", "p_ge_dbl", "p_ge_add_zone", "p_fe_mul", "p_fe_sq")
# opcodes the ubench does not time, priced as the measured opcode of the same encoding and width
ALIAS = {"v_addc_co_u32_e64": "v_addc_co_u32", "v_mov_b32_e32": "v_mov_b32", "v_mov_b64_e32": "v_mov_b64",
         "v_add_co_u32_e32": "v_add_co_u32", "v_add_co_u32_e64": "v_add_co_u32", "v_cmp_eq_u32_e32": "v_cmp_eq_u32",
         "v_lshlrev_b32_e32": "v_lshlrev_b32", "v_bfrev_b32_e32": "v_not_b32", "v_subb_co_u32_e32": "v_subb_co_u32",
         "v_sub_co_u32_e32": "v_sub_co_u32", "v_add_u32_e32": "v_add_u32", "v_max_u32_e32": "v_max_u32",
         "v_not_b32_e32": "v_not_b32", "v_or_b32_e32": "v_add_u32", "v_and_b32_e32": "v_add_u32",
         "v_xor_b32_e32": "v_add_u32", "v_cndmask_b32_e64": "v_cndmask_b32"}


def mixes():
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "ops.s")
        subprocess.run(["hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-S", "--cuda-device-only",
                        os.path.join(HERE, "isa_ops.hip"), "-o", out], check=True, stderr=subprocess.DEVNULL)
        s = open(out).read()
    res = {}
    for name in PROBES:
        body = s[s.index("\n" + name + ":"):]
        body = body[:body.index("s_endpgm")]
        ins, skip = [], False
        for l in body.split("\n"):
            t = l.strip()
            if skip:
                skip = t != "4:"
                continue
            if t == "s_branch 4f":   # the field asm's exact forms for rare edges: not the common path
                skip = True
                continue
            if l.startswith("\t") and t and not l.startswith("\t.") and not l.startswith("\t;"):
                ins.append(t.split()[0])
        res[name] = collections.Counter(i for i in ins if i.startswith("v_"))
    return res


def main():
    costs = json.load(open(sys.argv[1]))
    ops = costs["ops"]
    price = lambda op: ops[ALIAS.get(op, op)]["cycles"] if ALIAS.get(op, op) in ops else None
    out = {"source": os.path.relpath(sys.argv[1], ROOT), "device": costs.get("device"), "per_kernel": {}}
    for name, mix in mixes().items():
        n = sum(mix.values())
        known = {op: c for op, c in mix.items() if price(op) is not None}
        cyc = sum(price(op) * c for op, c in known.items())
        unpriced = {op: c for op, c in mix.items() if op not in known}
        # unpriced opcodes (few) take the mean price of the priced ones
        mean = cyc / sum(known.values())
        out["per_kernel"][name] = {"valu": n, "cycles": cyc + mean * sum(unpriced.values()),
                                   "cycles_per_valu": (cyc + mean * sum(unpriced.values())) / n,
                                   "unpriced": unpriced, "mix": dict(mix.most_common())}
    main_k = "p_ge_add_sel_zone"
    out["mix_kernel"] = main_k + " (the per-lane unified ge25519_add step with Z2 = 1: k_terms' dominant loop)"
    out["cycles_per_valu"] = out["per_kernel"][main_k]["cycles_per_valu"]
    path = os.path.join(ROOT, "profiles", "valu_issue_model.json")
    json.dump(out, open(path, "w"), indent=1)
    for k, v in out["per_kernel"].items():
        print(f"{k:20s} VALU {v['valu']:5d}  cycles {v['cycles']:8.1f}  cycles/VALU {v['cycles_per_valu']:.3f}  "
              f"unpriced {v['unpriced']}")


if __name__ == "__main__":
    main()
