"""The committed inline-asm headers are exactly what their generators emit (tools/gen_mul_asm.py ->
csrc/mul512_asm.h, tools/gen_field_asm.py -> csrc/field_asm.h), so a reviewer can read the
generator (with its hazard scheduling and the rare-edge tests) instead of the asm."""
import importlib.util
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _regen(tool, header, tmp_path):
    spec = importlib.util.spec_from_file_location(tool, os.path.join(ROOT, "tools", tool + ".py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    out = tmp_path / header
    mod.main(str(out))
    return out.read_text(), open(os.path.join(ROOT, "cudabulletproof_amd", "csrc", header)).read()


def test_mul_asm_header_is_generated(tmp_path):
    got, committed = _regen("gen_mul_asm", "mul512_asm.h", tmp_path)
    assert got == committed


def test_field_asm_header_is_generated(tmp_path):
    got, committed = _regen("gen_field_asm", "field_asm.h", tmp_path)
    assert got == committed
    # every exact form is reachable only through a rare-edge test: add, sub, fold and addsub as a
    # second asm statement under a C branch on the fast statement's srare (placed out of line by the
    # compiler); canon (cold) inline, branched over
    assert committed.count("s_cbranch_scc1") == 1
    assert committed.count("if (__builtin_expect(srare != 0, 0))") == 4 + 3   # + the latency forms of add, fold, addsub


def test_mul_asm_bounded_forms_drop_first_carries():
    """The bounded products count every carry but each column's first: 63 - 14 = 49 carry counts
    for mul512 (columns 1..14), 27 - 12 = 15 for the square's off-diagonal half (columns 2..13),
    and 7 for the 2x8 rows (columns 1..7; column 8's carry is never counted: the partial is
    < 2^320), against 63 / 27 / 14 in the counting forms."""
    import re
    h = open(os.path.join(ROOT, "cudabulletproof_amd", "csrc", "mul512_asm.h")).read()

    def counts(fn):
        body = h[h.index(f"void {fn}("):]
        body = body[:body.index("\n}\n")]
        return len(re.findall(r"v_addc_co_u32 %\[c2\]", body)), len(re.findall(r"v_mad_u64_u32", body))
    assert counts("mul512_asm") == (63, 64) and counts("mul512_bounded_asm") == (49, 64)
    assert counts("sqr512_offdiag_asm") == (27, 28) and counts("sqr512_offdiag_bounded_asm") == (15, 28)
    assert counts("mul2x8_asm") == (14, 16) and counts("mul2x8_bounded_asm") == (7, 16)


import pytest  # noqa: E402


@pytest.mark.parametrize("fn,rows,counted", [("mul512_k_asm", 8, 16), ("mul2x8_k_asm", 2, 1)])
def test_mul_by_k_counts_only_possible_carries(fn, rows, counted):
    """The products by k, the curve constant of every point operation (mul512_k_asm: a * k;
    mul2x8_k_asm: a lane's two rows of fe_mul_q4(x, k)), count 16 of 64 and 1 of 16 carries: each
    column takes its products smallest k-word first and counts a product only when the column's
    running-sum bound (carry-in bound + the products so far, every a word <= 2^32 - 1) can reach 2^64.
    Replayed here from the emitted asm, product by product: for the all-ones a (which maximises every
    partial sum, so it covers every input) and random a, no uncounted product overflows the 64-bit
    accumulator, and the replayed columns give the exact integer product a * k."""
    import random
    import re
    h = open(os.path.join(ROOT, "cudabulletproof_amd", "csrc", "mul512_asm.h")).read()
    body = h[h.index(f"void {fn}("):]
    body = body[:body.index("\n}\n")]
    kw = [int(x, 16) for x in re.search(r"kw\[8\] = \{([^}]*)\}", body).group(1).replace("u", "").split(",")]
    cols = []   # per column: [(i, j, counted)]
    for stmt in re.findall(r'asm volatile\("([^"]*)"', body):   # (column 0: one product onto 0, nothing counted)
        cols.append([(int(a), int(b), c != "sd" and bool(cols)) for c, a, b in
                     re.findall(r"v_mad_u64_u32 %\[acc\], %\[(\w+)\], %\[a(\d)\], %\[b(\d)\]", stmt)])
    assert len(cols) == rows + 7 and sum(len(c) for c in cols) == 8 * rows
    assert sum(c for col in cols for _, _, c in col) == counted == len(re.findall(r"v_addc_co_u32 %\[c2\]", body))
    K = sum(w << (32 * j) for j, w in enumerate(kw))
    rng = random.Random(5)
    for trial in range(2000):
        a = [0xFFFFFFFF] * rows if trial == 0 else [rng.choice([0xFFFFFFFF, rng.getrandbits(32)]) for _ in range(rows)]
        cin, words = 0, []
        for col in cols:
            acc, c2 = cin, 0
            for i, j, cnt in col:
                acc += a[i] * kw[j]
                if acc >= 2**64:
                    assert cnt, (trial, i, j)   # an uncounted product overflowed
                    acc -= 2**64
                    c2 += 1
            words.append(acc & 0xFFFFFFFF)
            cin = (acc >> 32) + (c2 << 32)
        words.append(cin & 0xFFFFFFFF)
        assert cin >> 32 == 0
        A = sum(w << (32 * i) for i, w in enumerate(a))
        assert sum(w << (32 * k) for k, w in enumerate(words)) == A * K


def _asm_statements(path):
    """Every inline-asm text of a generated header, split into instruction lines."""
    s = open(path).read()
    out = []
    for m in re.finditer(r'asm volatile\("((?:[^"\\]|\\.)*)"', s):
        out.append([t.strip() for t in m.group(1).replace("\\n", "\n").replace("\\t", "").split("\n") if t.strip()])
    return out


def _operands(line):
    op, _, rest = line.partition(" ")
    return op, [x.strip() for x in rest.split(",")] if rest else []


def test_generated_asm_hazard_spacing():
    """Inside every generated asm statement (mul512_asm.h, field_asm.h), on each straight-line
    segment: an SGPR a VALU instruction writes is read as a carry-in no sooner than 1 wait state
    later and as a mask (v_cndmask) no sooner than 2; a VGPR a VALU instruction writes is read by a
    DPP move no sooner than 2 (intervening instructions count 1 each, s_nop N counts N + 1).  A label
    starts a new segment (its state comes from several predecessors: the generator's scheduler merges
    them; here only reads of registers written in the same segment are checked)."""
    import os
    root = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "cudabulletproof_amd", "csrc")
    carry_ops = ("v_addc_co_u32", "v_subb_co_u32", "v_subbrev_co_u32")
    checked = 0
    for hdr in ("mul512_asm.h", "field_asm.h"):
        for lines in _asm_statements(os.path.join(root, hdr)):
            sgpr_w, vgpr_w, pos = {}, {}, 0
            for line in lines:
                if line.endswith(":"):   # a label: a new segment
                    sgpr_w, vgpr_w = {}, {}
                    continue
                op, ops = _operands(line)
                if op == "s_nop":
                    pos += int(ops[0]) + 1
                    continue
                if op.startswith("v_"):
                    reads = ops[1:]
                    if op.startswith("v_mov_b32_dpp"):
                        src = reads[0].split()[0]
                        if src in vgpr_w:
                            assert pos - vgpr_w[src] - 1 >= 2, (hdr, line)
                            checked += 1
                    if op in carry_ops and reads and reads[-1] in sgpr_w:
                        assert pos - sgpr_w[reads[-1]] - 1 >= 1, (hdr, line)
                        checked += 1
                    if op.startswith("v_cndmask") and reads and reads[-1] in sgpr_w:
                        assert pos - sgpr_w[reads[-1]] - 1 >= 2, (hdr, line)
                        checked += 1
                    if op in ("v_add_co_u32", "v_sub_co_u32", "v_mad_u64_u32") + carry_ops or op.startswith("v_cmp"):
                        sdst = ops[1] if not op.startswith("v_cmp") else ops[0]
                        sgpr_w[sdst] = pos
                    vgpr_w[ops[0]] = pos
                elif op.startswith("s_") and ops:
                    sgpr_w.pop(ops[0], None)   # a SALU write: readable at once
                if op.startswith(("s_branch", "s_cbranch")):
                    sgpr_w, vgpr_w = {}, {}
                pos += 1
    assert checked > 250, checked   # (315 reads checked at round 6)


def test_deferred_forms_are_the_fast_statements():
    """field_asm.h's *_lat_acc forms (the row step's deferred rare-edge test) are their *_lat block's
    fast statement with the one rare-edge compare replaced by the running max into acc: the same
    instructions otherwise, so the same results, and the same test words feed the deferred test."""
    s = open(os.path.join(ROOT, "cudabulletproof_amd", "csrc", "field_asm.h")).read()

    def statements(fn):
        body = s[s.index(f"void {fn}("):]
        body = body[:body.index("\n}\n")]
        return [m.group(1) for m in re.finditer(r'asm volatile\("((?:[^"\\]|\\.)*)"', body)]
    for fn in ("fe_add_asm_lat", "fe_fold_asm_lat", "fe_addsub_asm_lat"):
        fast = statements(fn)[0]
        acc = statements(fn + "_acc")
        assert len(acc) == 1 and fast.count("v_cmp_eq_u32 %[srare], -1, %[vt3]") == 1
        assert acc[0] == fast.replace("v_cmp_eq_u32 %[srare], -1, %[vt3]", "v_max_u32 %[acc], %[acc], %[vt3]")
