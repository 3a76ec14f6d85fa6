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
    assert committed.count("s_cbranch_scc1") == 2 + 1 + 2 + 1 + 1   # sub 2, add 1, fold 2, canon 1, addsub 1
