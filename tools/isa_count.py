"""Compile tools/isa_ops.hip for gfx950 and print per-kernel VALU / s_nop counts.

  python tools/isa_count.py [extra hipcc flags]
"""
import collections
import os
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))


def main():
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "ops.s")
        subprocess.run(["hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-S", "--cuda-device-only",
                        os.path.join(HERE, "isa_ops.hip"), "-o", out] + sys.argv[1:], check=True)
        s = open(out).read()
    for name in [l.split(":")[0] for l in s.split("\n") if l.startswith("p_") and l.split(":")[0].isidentifier()]:
        body = s[s.index("\n" + name + ":"):]
        body = body[:body.index("s_endpgm")]
        ins = [l.split()[0] for l in body.split("\n")
               if l.startswith("\t") and l.strip() and not l.startswith("\t.") and not l.startswith("\t;")]
        c = collections.Counter(ins)
        valu = sum(n for i, n in c.items() if i.startswith("v_"))
        top = ", ".join(f"{k}:{v}" for k, v in c.most_common(8))
        print(f"{name:14s} VALU {valu:5d}  s_nop {c['s_nop']:4d}  SALU {sum(n for i, n in c.items() if i.startswith('s_') and i != 's_nop'):4d}  | {top}")


if __name__ == "__main__":
    main()
