"""Compile tools/isa_ops.hip for gfx950 and print per-kernel VALU / s_nop counts (common path:
the field asm's exact forms for rare edges are skipped).

  python tools/isa_count.py [extra hipcc flags]
"""
import collections
import re
import os
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))

# issue cost per wave64 instruction, cycles at 8 waves/SIMD (tools/ubench_enc.hip on MI355X, nominal clock)
FULL = ("v_add_u32", "v_sub_u32", "v_and_b32", "v_or_b32", "v_xor_b32", "v_mov_b32", "v_not_b32", "v_subrev_u32")


def cost(op):
    base = op.split("_e32")[0].split("_e64")[0]
    if base in FULL:
        return 2.4
    if base == "v_mad_u64_u32":
        return 5.1
    if base in ("v_lshl_add_u64",):
        return 4.7
    if base.startswith("v_"):
        return 4.5
    return 0.0


def main():
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "ops.s")
        subprocess.run(["hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-S", "--cuda-device-only",
                        os.path.join(HERE, "isa_ops.hip"), "-o", out] + sys.argv[1:], check=True)
        s = open(out).read()
    for name in [l.split(":")[0] for l in s.split("\n") if l.startswith("p_") and l.split(":")[0].isidentifier()]:
        body = s[s.index("\n" + name + ":"):]
        body = body[:body.index("s_endpgm")]
        if name.startswith("p_sm_"):   # a loop kernel: the last backward branch's body (one iteration)
            lines = body.split("\n")
            labels = {l.split(":")[0]: i for i, l in enumerate(lines) if re.match(r"^\.LBB\d+_\d+:", l)}
            span = None
            for i, l in enumerate(lines):
                m = re.search(r"s_(?:cbranch_\w+|branch)\s+(\.LBB\d+_\d+)", l)
                if m and m.group(1) in labels and labels[m.group(1)] < i:
                    span = (labels[m.group(1)], i)
            if span:
                body = "\n".join(lines[span[0]:span[1] + 1])
                name += " (loop body)"
        # the field asm's exact forms for rare edges sit between "s_branch 4f" and the "4:" label:
        # count the common path only (what a wave executes unless a lane is on a rare edge)
        ins, skip = [], False
        for l in body.split("\n"):
            t = l.strip()
            if skip:
                skip = t != "4:"
                continue
            if t == "s_branch 4f":
                skip = True
                ins.append("s_branch")
                continue
            if l.startswith("\t") and t and not l.startswith("\t.") and not l.startswith("\t;"):
                ins.append(t.split()[0])
        c = collections.Counter(ins)
        valu = sum(n for i, n in c.items() if i.startswith("v_"))
        top = ", ".join(f"{k}:{v}" for k, v in c.most_common(8))
        cyc = sum(cost(i) * n for i, n in c.items() if not i.startswith(("global_", "ds_", "buffer_", "scratch_")))
        print(f"{name:14s} VALU {valu:5d}  ~cyc {cyc:7.0f}  s_nop {c['s_nop']:4d}  "
              f"SALU {sum(n for i, n in c.items() if i.startswith('s_') and i != 's_nop'):4d}  | {top}")
        if os.environ.get("ISA_FULL") and os.environ["ISA_FULL"] in name:   # every VALU opcode of one kernel
            print("    " + ", ".join(f"{k}:{v}" for k, v in sorted(c.items(), key=lambda kv: -kv[1]) if k.startswith("v_")))


if __name__ == "__main__":
    main()
