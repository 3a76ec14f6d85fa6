"""The committed inline-asm headers are exactly what their generators emit (tools/gen_mul_asm.py ->
csrc/mul512_asm.h, tools/gen_field_asm.py -> csrc/field_asm.h), so a reviewer can read the
generator (with its hazard scheduling and the rare-edge tests) instead of the asm."""
import importlib.util
import os

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
    # every exact form is reachable only through a rare-edge test and rejoins at the end
    assert committed.count("s_cbranch_scc1") == 2 + 1 + 1 + 1 + 1   # sub 2, add 1, fold 1, canon 1, addsub 1


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
