"""Generate cudabulletproof_amd/csrc/field_asm.h: gfx950 inline-asm forms of the reference's
lossy field add / product fold (curve25519_ops.cu:41-146), SAME bits as the C forms in
fe25519_dev.h (which stay the host-pass / reference formulation).

Why asm: the fix-up "(carry || h >= p) ? lossy - p : h" is a data-dependent select.  Written in
C the compiler materialises each mask with v_cmp + v_cndmask (4.5-4.6 cycles per wave
instruction, tools/ubench_enc.hip) and adds through 64-bit v_lshl_add_u64 (4.7); here the masks
stay in SGPRs, are combined by SALU (its own issue port) and enter the arithmetic as the carry-ins
of v_addc.  Every operand is a 32-bit VGPR: the C side passes limb halves (free sub-registers),
so no register pair has to be formed.

Hazard rule these sequences meet (gfx950): an SGPR written by a VALU instruction (carry-out,
v_cmp) and read by a VALU instruction as a mask or source operand (v_cndmask) needs 2 wait states
in between, read as a carry-in (v_addc / v_subb) 1 wait state, the spacing the compiler itself
gives the same e64 carry chains (tools/hazard_probe.hip read no stale carry even at 0 on MI355X);
SALU-written masks can be read at once.  `schedule` inserts the s_nop.  Outputs are VGPRs only,
inputs are VGPRs or constants, so nothing crosses the asm boundary in an SGPR.
"""
import os

HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(HERE, "..", "cudabulletproof_amd", "csrc", "field_asm.h")
GUARD = []       # no trailing wait states: see emit()
WAIT_MASK = 2    # VALU-written SGPR read as a mask / source operand
WAIT_CARRY = 1   # ... read as the carry-in of v_addc / v_subb
CARRY_READERS = ("v_addc_co_u32", "v_subb_co_u32", "v_subbrev_co_u32")


def schedule(ins, state=None):
    """ins: (text, sgpr_writes, sgpr_reads, is_valu).  Returns the lines with s_nop inserted and the
    end state {sgpr: wait states since its VALU write}.  `state` carries the predecessors' end
    state into a segment (branch targets: the merged, most recent writes)."""
    lines, pos, wpos = [], 0, {}
    for r, d in (state or {}).items():
        wpos[r] = -1 - d
    for text, writes, reads, is_valu in ins:
        if is_valu:
            need = 0
            wait = WAIT_CARRY if text.split()[0] in CARRY_READERS else WAIT_MASK
            for r in reads:
                if r in wpos:
                    need = max(need, wait - (pos - wpos[r] - 1))
            if need > 0:
                lines.append(f"s_nop {need - 1}")
                pos += need
        lines.append(text)
        for w in writes:
            if is_valu:
                wpos[w] = pos
            else:
                wpos.pop(w, None)
        pos += 1
    return lines, {r: pos - p - 1 for r, p in wpos.items()}


def merge(*states):
    out = {}
    for st in states:
        for r, d in st.items():
            out[r] = min(d, out.get(r, d))
    return out


def V(t, w=(), r=()):
    return (t, list(w), list(r), True)


def S(t, w=()):
    return (t, list(w), [], False)


def cref(carry):
    """carry-out mask operand: an SGPR pair name, or the literal 0 (no carry)."""
    return "0" if carry == "0" else f"%[{carry}]"


def fix_seq(h, o, carry):
    """(carry || h >= p) ? lossy "- p" : h (curve25519_ops.cu:54-66), halves h[0..7] -> o[0..7].
    m = carry | top | (h3 == P3 & h2 == M & h1 == M & h0 >= P0);
    out_i = h_i + m * (19, !br1, !br2, 2^63 + !br3)_i, no carries between limbs, with
    br1 = h0 < P0, br2 = !br1 & h1 != M, br3 = !br2 & h2 != M (fe25519_dev.h fe_fix)."""
    q = [V(f"v_and_b32 %[vt1], %[{h[2]}], %[{h[3]}]"),
         V(f"v_and_b32 %[vt2], %[{h[4]}], %[{h[5]}]"),
         V(f"v_or_b32 %[vt3], %[c80], %[{h[7]}]"),
         V("v_cmp_eq_u32 %[sf1], -1, %[vt1]", ["sf1"]),                   # h1 == M
         V("v_cmp_eq_u32 %[sf2], -1, %[vt2]", ["sf2"]),                   # h2 == M
         V(f"v_and_b32 %[vt3], %[vt3], %[{h[6]}]"),
         V("v_cmp_eq_u32 %[se3], -1, %[vt3]", ["se3"]),                   # h3 == P3 (or M: top set too)
         V(f"v_cmp_gt_i32 %[stp], 0, %[{h[7]}]", ["stp"]),                # bit 255
         V(f"v_cmp_eq_u32 %[sg0], -1, %[{h[1]}]", ["sg0"]),
         V(f"v_cmp_le_u32 %[sg1], %[p0l], %[{h[0]}]", ["sg1"]),
         S("s_and_b64 %[sg0], %[sg0], %[sg1]", ["sg0"]),                  # ge0 = h0 >= P0 = !br1
         S("s_and_b64 %[se3], %[se3], %[sf1]", ["se3"]),
         S("s_and_b64 %[se3], %[se3], %[sf2]", ["se3"]),
         S("s_and_b64 %[se3], %[se3], %[sg0]", ["se3"]),
         S(f"s_or_b64 %[sm], {cref(carry)}, %[stp]", ["sm"]),
         S("s_or_b64 %[sm], %[sm], %[se3]", ["sm"]),                      # m
         S("s_and_b64 %[sd1], %[sm], %[sg0]", ["sd1"]),                   # m & !br1
         S("s_orn2_b64 %[sg1], %[sf1], %[sg0]", ["sg1"]),                 # !br2 = f1 | !ge0
         S("s_and_b64 %[sd2], %[sm], %[sg1]", ["sd2"]),                   # m & !br2
         S("s_andn2_b64 %[sg1], %[sg0], %[sf1]", ["sg1"]),                # br2 = ge0 & !f1
         S("s_or_b64 %[sg1], %[sg1], %[sf2]", ["sg1"]),                   # !br3 = br2 | f2
         S("s_and_b64 %[sd3], %[sm], %[sg1]", ["sd3"]),                   # m & !br3
         V("v_cndmask_b32 %[vt1], 0, 19, %[sm]", [], ["sm"]),
         V("v_cndmask_b32 %[vt2], 0, %[c80], %[sm]", [], ["sm"]),
         V(f"v_add_co_u32 %[{o[0]}], %[sk0], %[{h[0]}], %[vt1]", ["sk0"]),
         V(f"v_addc_co_u32 %[{o[2]}], %[sk1], %[{h[2]}], 0, %[sd1]", ["sk1"], ["sd1"]),
         V(f"v_addc_co_u32 %[{o[4]}], %[sk2], %[{h[4]}], 0, %[sd2]", ["sk2"], ["sd2"]),
         V(f"v_addc_co_u32 %[{o[6]}], %[sk3], %[{h[6]}], 0, %[sd3]", ["sk3"], ["sd3"]),
         V(f"v_addc_co_u32 %[{o[1]}], %[sk0], %[{h[1]}], 0, %[sk0]", ["sk0"], ["sk0"]),
         V(f"v_addc_co_u32 %[{o[3]}], %[sk1], %[{h[3]}], 0, %[sk1]", ["sk1"], ["sk1"]),
         V(f"v_addc_co_u32 %[{o[5]}], %[sk2], %[{h[5]}], 0, %[sk2]", ["sk2"], ["sk2"]),
         V(f"v_addc_co_u32 %[{o[7]}], %[sk3], %[{h[7]}], %[vt2], %[sk3]", ["sk3"], ["sk3"])]
    return q


FIX_SGPRS = ["sf1", "sf2", "se3", "stp", "sg0", "sg1", "sm", "sd1", "sd2", "sd3", "sk0", "sk1", "sk2", "sk3"]


def fix_test(h, carry):
    """Wave-uniform test for fix_seq's fast form.  With h0 < P0 (br1 = 1) the fix-up's m is
    carry | top (the equality case needs h0 >= P0), br2 = 0 and br3 = !(h2 == M), so when also
    h2 != M every lane's result is h + m (19, 0, 1, 2^63).  h0 >= P0 implies h0's high word is
    2^32-1 and h2 == M implies its low word is: srare = max(those words) == 2^32-1 is a superset of
    the lanes that need the exact form.  Also forms m = carry | top in sm."""
    return [V(f"v_max_u32 %[vt3], %[{h[1]}], %[{h[4]}]"),
            V(f"v_cmp_gt_i32 %[stp], 0, %[{h[7]}]", ["stp"]),
            V("v_cmp_eq_u32 %[srare], -1, %[vt3]", ["srare"]),
            S(f"s_or_b64 %[sm], {cref(carry)}, %[stp]", ["sm"])]


def fix_fast(h):
    """h += m (19, 0, 1, 2^63) per limb, in place (valid when fix_test found no rare lane)."""
    return [V("v_cndmask_b32 %[vt1], 0, 19, %[sm]", [], ["sm"]),
            V("v_cndmask_b32 %[vt2], 0, %[c80], %[sm]", [], ["sm"]),
            V(f"v_add_co_u32 %[{h[0]}], %[sk0], %[{h[0]}], %[vt1]", ["sk0"]),
            V(f"v_addc_co_u32 %[{h[4]}], %[sk2], %[{h[4]}], 0, %[sm]", ["sk2"], ["sm"]),
            V(f"v_add_u32 %[{h[7]}], %[{h[7]}], %[vt2]"),
            V(f"v_addc_co_u32 %[{h[1]}], %[sk0], %[{h[1]}], 0, %[sk0]", ["sk0"], ["sk0"]),
            V(f"v_addc_co_u32 %[{h[5]}], %[sk2], %[{h[5]}], 0, %[sk2]", ["sk2"], ["sk2"])]


def fix_fast_lat(h, carry="scy"):
    """fix_fast for the latency forms (the 16-lane row step): m = carry | top as a VALU mask, 0 or
    -1, instead of a compare and the SALU OR, which waits ≈16 cycles on that compare when one wave
    runs alone (tools/ubench_dep.hip cmp_sor_add).  Two more VALU than fix_fast's compare and two
    selects: a loss where many waves hide the wait (the throughput kernels keep fix_fast)."""
    return [V(f"v_ashrrev_i32 %[vt2], 31, %[{h[7]}]"),
            V(f"v_cndmask_b32 %[vt2], %[vt2], -1, %[{carry}]", [], [carry]),
            V("v_and_b32 %[vt1], 19, %[vt2]"),
            V("v_lshrrev_b32 %[vt3], 31, %[vt2]"),
            V("v_and_b32 %[vt2], %[c80], %[vt2]"),
            V(f"v_add_co_u32 %[{h[0]}], %[sk0], %[{h[0]}], %[vt1]", ["sk0"]),
            V(f"v_add_co_u32 %[{h[4]}], %[sk2], %[{h[4]}], %[vt3]", ["sk2"]),
            V(f"v_add_u32 %[{h[7]}], %[{h[7]}], %[vt2]"),
            V(f"v_addc_co_u32 %[{h[1]}], %[sk0], %[{h[1]}], 0, %[sk0]", ["sk0"], ["sk0"]),
            V(f"v_addc_co_u32 %[{h[5]}], %[sk2], %[{h[5]}], 0, %[sk2]", ["sk2"], ["sk2"])]


def branch_if_rare(label):
    return [S("s_cmp_lg_u64 %[srare], 0"), S(f"s_cbranch_scc1 {label}")]


def emit(name, doc, args, ins, outs, vtemps, sgprs, lines, inout=False):
    """args: [(param, prefix)] array params bound to scalars prefix0..7.  lines: scheduled asm.
    inout: the outputs are read-write, initialised from the first array argument."""
    # No trailing wait states (rounds 2-6 ended every block with s_nop 4 against "a VALU SGPR write
    # followed by a VMEM read of it needs 5").  The block's SGPR outputs are early-clobber temporaries
    # that nothing reads after it, so any later read of those registers follows a new write of them
    # (the compiler's own, which it pads itself); tools/asm_exit_check.py scans every compiled kernel
    # for a memory instruction reading an SGPR the block wrote within 5 states (none).
    text = "\\n\\t".join(lines + GUARD)
    out = [f"// {d}" for d in doc]
    out.append(f"__device__ __forceinline__ void {name}(uint32_t out[8], " +
               ", ".join(f"const uint32_t {p}[8]" for p, _ in args) + ") {")
    if inout:
        out.append("    uint32_t " + ", ".join(f"{x} = {args[0][0]}[{i}]" for i, x in enumerate(outs)) + ";")
        out.append("    uint32_t " + ", ".join(vtemps) + ";")
    else:
        for p, pre in args:
            out.append("    const uint32_t " + ", ".join(f"{pre}{i} = {p}[{i}]" for i in range(8)) + ";")
        out.append("    uint32_t " + ", ".join(outs + vtemps) + ";")
    out.append("    uint64_t " + ", ".join(sgprs) + ";")
    out.append(f'    asm volatile("{text}"')
    out.append("                 : " + ", ".join([f'[{x}] "{"+v" if inout else "=&v"}"({x})' for x in outs] +
                                          [f'[{x}] "=&v"({x})' for x in vtemps] +
                                          [f'[{x}] "=&s"({x})' for x in sgprs]))
    out.append("                 : " + ", ".join([f'[{x}] "v"({x})' for x in ins] +
                                          ['[c80] "v"(0x80000000u)', '[p0l] "s"(0xFFFFFFEDu)']))
    # the SALU mask logic overwrites SCC; without the clobber the compiler keeps a compare's SCC
    # live across the block (seen: s_cmp before the block, s_cbranch_scc1 after it)
    out.append('                 : "scc");')
    for i in range(8):
        out.append(f"    out[{i}] = {outs[i]};")
    out.append("    (void)" + "; (void)".join(sgprs + vtemps) + ";")
    out.append("}")
    return out


def two_way(pre, fast, slow):
    """pre; if any lane is rare: slow, else fast (wave-uniform branch on srare, set in pre).
    Layout: pre, branch, fast, s_branch to the end, slow (label 3), end (label 4)."""
    lp, sp = schedule(pre + branch_if_rare("3f"))
    lf, sf = schedule(fast, sp)
    ls, ss = schedule(slow, sp)
    _, _ = merge(sf, ss), None
    return lp + lf + ["s_branch 4f", "3:"] + ls + ["4:"]


def emit_split(name, doc, args, outs, vtemps, fast_sgprs, fast, slow_sgprs, slow):
    """The fast form and the exact form as two asm statements: the fast one computes the common result
    and the wave-uniform rare-edge mask srare; the exact one (from the inputs again) runs under a C
    branch the compiler places out of line.  Measured on one wave (tools/ubench_dep.hip,
    profiles/ubench/ubench_dep_r06.json): a compare read by the SALU test right after it stalls the
    wave ~20 cycles and the taken s_branch over an inline exact form costs ~22; srare is written
    early in the fast statement, so the test after it finds it ready, and the common path falls
    through (a not-taken branch, ~8 cycles)."""
    ins = [f"{pre}{i}" for _, pre in args for i in range(8)]
    outs_c = [f'[{x}] "=&v"({x})' for x in outs + vtemps]
    ins_c = ", ".join([f'[{x}] "v"({x})' for x in ins] + ['[c80] "v"(0x80000000u)', '[p0l] "s"(0xFFFFFFEDu)'])
    out = [f"// {d}" for d in doc]
    out.append(f"__device__ __forceinline__ void {name}(" + ", ".join(f"uint32_t o{k}[8]" for k in range(len(outs) // 8)) +
               ", " + ", ".join(f"const uint32_t {p}[8]" for p, _ in args) + ") {")
    for p, pre in args:
        out.append("    const uint32_t " + ", ".join(f"{pre}{i} = {p}[{i}]" for i in range(8)) + ";")
    out.append("    uint32_t " + ", ".join(outs + vtemps) + ";")
    out.append("    uint64_t " + ", ".join(fast_sgprs) + ";")
    out.append('    asm volatile("{0}"'.format("\\n\\t".join(fast)))
    out.append("                 : " + ", ".join(outs_c + [f'[{x}] "=&s"({x})' for x in fast_sgprs]))
    out.append("                 : " + ins_c)
    out.append('                 : "scc");')
    out.append("    if (__builtin_expect(srare != 0, 0)) {   // some lane is on a rare edge: the exact form")
    out.append("        uint64_t " + ", ".join(slow_sgprs) + ";")
    out.append('        asm volatile("{0}"'.format("\\n\\t".join(slow)))
    out.append("                     : " + ", ".join(outs_c + [f'[{x}] "=&s"({x})' for x in slow_sgprs]))
    out.append("                     : " + ins_c)
    out.append('                     : "scc");')
    out.append("        (void)" + "; (void)".join(slow_sgprs) + ";")
    out.append("    }")
    for k in range(len(outs) // 8):
        out.append("    " + " ".join(f"o{k}[{i}] = {outs[8 * k + i]};" for i in range(8)))
    out.append("    (void)" + "; (void)".join(fast_sgprs + vtemps) + ";")
    out.append("}")
    return out


def emit_acc(name, doc, args, outs, vtemps, sgprs, fast):
    """The fast statement alone, for callers that defer the rare-edge test (the row step): the words
    the test reads go into the caller's running max `acc` (v_max_u32 in place of the compare); a
    rare lane shows as acc == 2^32-1 and the caller recomputes the whole step with the exact-capable
    forms.  Same VALU count as the fast statement of emit_split, no SALU test, no branch."""
    ins = [f"{pre}{i}" for _, pre in args for i in range(8)]
    out = [f"// {d}" for d in doc]
    out.append(f"__device__ __forceinline__ void {name}(" + ", ".join(f"uint32_t o{k}[8]" for k in range(len(outs) // 8)) +
               ", " + ", ".join(f"const uint32_t {p}[8]" for p, _ in args) + ", uint32_t& acc) {")
    for p, pre in args:
        out.append("    const uint32_t " + ", ".join(f"{pre}{i} = {p}[{i}]" for i in range(8)) + ";")
    out.append("    uint32_t " + ", ".join(outs + vtemps) + ";")
    out.append("    uint64_t " + ", ".join(sgprs) + ";")
    out.append('    asm volatile("{0}"'.format("\\n\\t".join(fast)))
    out.append("                 : " + ", ".join([f'[{x}] "=&v"({x})' for x in outs + vtemps] + ['[acc] "+v"(acc)'] +
                                          [f'[{x}] "=&s"({x})' for x in sgprs]))
    out.append("                 : " + ", ".join([f'[{x}] "v"({x})' for x in ins] + ['[c80] "v"(0x80000000u)']))
    out.append('                 : "scc");')
    for k in range(len(outs) // 8):
        out.append("    " + " ".join(f"o{k}[{i}] = {outs[8 * k + i]};" for i in range(8)))
    out.append("    (void)" + "; (void)".join(sgprs + vtemps) + ";")
    out.append("}")
    return out


def to_acc(fast):
    """The fast statement with the rare-edge compare replaced by the running max into acc."""
    out = []
    for t in fast:
        if t[0] == "v_cmp_eq_u32 %[srare], -1, %[vt3]":
            out.append(V("v_max_u32 %[acc], %[acc], %[vt3]"))
        else:
            out.append(t)
    assert len(out) == len(fast) and any(t[0].startswith("v_max_u32 %[acc]") for t in out)
    return out


def add_chain(h, a="a", b="b", cy="scy", upto=8, start=0):
    out = []
    for i in range(start, upto):
        if i == 0:
            out.append(V(f"v_add_co_u32 %[{h[0]}], %[{cy}], %[{a}0], %[{b}0]", [cy]))
        else:
            out.append(V(f"v_addc_co_u32 %[{h[i]}], %[{cy}], %[{a}{i}], %[{b}{i}], %[{cy}]", [cy], [cy]))
    return out


def gen_add(lat=False, acc=False):
    """Fast statement: the add chain with fix_test's compare placed as soon as h1 and h4 exist, then
    m = carry | top and the fast fix-up (lat: fix_fast_lat).  Exact statement: the chain again and
    fix_seq."""
    h = [f"h{i}" for i in range(8)]
    fast = add_chain(h, upto=5) + [V("v_max_u32 %[vt3], %[h1], %[h4]"),
                                    V("v_cmp_eq_u32 %[srare], -1, %[vt3]", ["srare"])] + add_chain(h, start=5)
    if lat:
        fast += fix_fast_lat(h)
    else:
        fast += [V("v_cmp_gt_i32 %[stp], 0, %[h7]", ["stp"]), S("s_or_b64 %[sm], %[scy], %[stp]", ["sm"])] + fix_fast(h)
    lf, _ = schedule(fast)
    if acc:
        return emit_acc("fe_add_asm_lat_acc", ["fe_add_asm_lat's fast statement, the rare-edge test deferred into acc (emit_acc)."],
                        [("fa", "a"), ("ga", "b")], h, ["vt1", "vt2", "vt3"], ["scy", "sk0", "sk2"],
                        schedule(to_acc(fast))[0])
    ls, _ = schedule(add_chain(h) + fix_seq(h, h, "scy"))
    return emit_split("fe_add_asm" + ("_lat" if lat else ""), ["fe25519_add (curve25519_ops.cu:41-68) on limb halves: exact 257-bit sum, then",
                                     "one lossy \"- p\" when it carried out or is >= p (fast form unless a lane is",
                                     "on one of the fix-up's rare edges: fix_test)."],
                      [("fa", "a"), ("ga", "b")], h, ["vt1", "vt2", "vt3"],
                      ["scy", "srare", "sk0", "sk2"] + ([] if lat else ["stp", "sm"]), lf, FIX_SGPRS + ["scy"], ls)


def gen_fold(lat=False, acc=False):
    """One wave-uniform rare-edge test: if some x_i (i = 1..3) may be 2^64-1 (its low word is: the
    lossy carry can differ from the true one) or fix_test's edge words are all ones, the exact chain
    (from the inputs again) + exact fix-up; else the plain chain + the fast fix-up."""
    h = [f"h{i}" for i in range(8)]
    plain = [V("v_add_co_u32 %[h0], %[scy], %[a0], %[x0]", ["scy"])]
    for i in range(1, 8):
        plain.append(V(f"v_addc_co_u32 %[h{i}], %[scy], %[a{i}], %[x{i}], %[scy]", ["scy"], ["scy"]))
    exact = []
    for i in (1, 2, 3):   # x_i == 2^64-1 (limb 0 has no carry-in)
        exact.append(V(f"v_and_b32 %[vt1], %[x{2 * i}], %[x{2 * i + 1}]"))
        exact.append(V(f"v_cmp_eq_u32 %[sq{i}], -1, %[vt1]", [f"sq{i}"]))
    exact.append(V("v_add_co_u32 %[h0], %[sk0], %[a0], %[x0]", ["sk0"]))
    exact.append(V("v_addc_co_u32 %[h1], %[scy], %[a1], %[x1], %[sk0]", ["scy"], ["sk0"]))
    for i in (1, 2, 3):
        exact.append(V(f"v_addc_co_u32 %[h{2 * i}], %[sk0], %[a{2 * i}], %[x{2 * i}], %[scy]", ["sk0"], ["scy"]))
        exact.append(V(f"v_addc_co_u32 %[h{2 * i + 1}], %[sk1], %[a{2 * i + 1}], %[x{2 * i + 1}], %[sk0]",
                       ["sk1"], ["sk0"]))
        exact.append(S(f"s_and_b64 %[sq{i}], %[sq{i}], %[scy]", [f"sq{i}"]))   # x_i == M & carry-in
        exact.append(S(f"s_andn2_b64 %[scy], %[sk1], %[sq{i}]", ["scy"]))      # the reference's carry
    # fast statement: the x words' max first, the chain, the h words' max and the one compare as soon
    # as h1 and h4 exist, the rest of the chain, m = carry | top, the fast fix-up.  Exact statement:
    # the exact chain from the inputs again and the exact fix-up.
    fast = [V("v_max3_u32 %[vt3], %[x2], %[x4], %[x6]")] + plain[:5] + \
        [V(f"v_max3_u32 %[vt3], %[vt3], %[{h[1]}], %[{h[4]}]"),
         V("v_cmp_eq_u32 %[srare], -1, %[vt3]", ["srare"])] + plain[5:]
    if lat:
        fast += fix_fast_lat(h)
    else:
        fast += [V(f"v_cmp_gt_i32 %[stp], 0, %[{h[7]}]", ["stp"]),
                 S(f"s_or_b64 %[sm], {cref('scy')}, %[stp]", ["sm"])] + fix_fast(h)
    lf, _ = schedule(fast)
    if acc:
        return emit_acc("fe_fold_asm_lat_acc", ["fe_fold_asm_lat's fast statement, the rare-edge test deferred into acc (emit_acc)."],
                        [("ta", "a"), ("xa", "x")], h, ["vt1", "vt2", "vt3"], ["scy", "sk0", "sk2"],
                        schedule(to_acc(fast))[0])
    ls, _ = schedule(exact + fix_seq(h, h, "scy"))
    return emit_split("fe_fold_asm" + ("_lat" if lat else ""), ["Fold of the exact 512-bit product (curve25519_ops.cu:114-145): t_lo as halves",
                                      "ta[0..7], x_i = lo64(19 t_{i+4}) as halves xa[0..7]; carry chain with the lossy",
                                      "carry cy_i = c_i & !(x_i == 2^64-1 & cy_{i-1}), then the fix-up.  The plain",
                                      "chain and the fast fix-up unless a lane is on a rare edge (wave-uniform test)."],
                      [("ta", "a"), ("xa", "x")], h, ["vt1", "vt2", "vt3"],
                      ["scy", "srare", "sk0", "sk2"] + ([] if lat else ["stp", "sm"]), lf,
                      FIX_SGPRS + ["scy", "sq1", "sq2", "sq3"], ls)


def gen_sub():
    """fe25519_sub (curve25519_ops.cu:71-90): t = f - g with the lossy borrow
    br_i = b_i & !(g_i == 2^64-1 & br_{i-1}); on a final borrow m, the literal "+ p" pass:
    o0 = t0 - 19m; o1 = t1 - (m & t0 < 19); o2 = t2 - (m & o1 == M); o3 = t3 + m 2^63 - (m & o2 == M)
    (fe25519_dev.h fe_sub).  m & t0 < 19 is exactly the borrow out of o0's subtraction.
    Fast form (wave-uniform tests): no lane's g_1..g_3 may be 2^64-1 (their low words are not),
    so the borrow chain is the plain one; and no lane has t0 < 19 (implies t0's high word is 0),
    t1 == M or t2 == M (their low words are 2^32-1), so the "+ p" pass is t + m (-19, 0, 0, 2^63)."""
    t = [f"h{i}" for i in range(8)]
    plain = [V("v_sub_co_u32 %[h0], %[scy], %[a0], %[b0]", ["scy"])]
    for i in range(1, 8):
        plain.append(V(f"v_subb_co_u32 %[h{i}], %[scy], %[a{i}], %[b{i}], %[scy]", ["scy"], ["scy"]))
    fastp = [V("v_cndmask_b32 %[vt1], 0, 19, %[scy]", [], ["scy"]),
             V("v_cndmask_b32 %[vt2], 0, %[c80], %[scy]", [], ["scy"]),
             V("v_sub_co_u32 %[h0], %[sk0], %[h0], %[vt1]", ["sk0"]),
             V("v_add_u32 %[h7], %[h7], %[vt2]"),
             V("v_subb_co_u32 %[h1], %[sk0], %[h1], 0, %[sk0]", ["sk0"], ["sk0"])]
    exact = []
    for i in (1, 2, 3):   # g_i == 2^64-1
        exact.append(V(f"v_and_b32 %[vt1], %[b{2 * i}], %[b{2 * i + 1}]"))
        exact.append(V(f"v_cmp_eq_u32 %[sq{i}], -1, %[vt1]", [f"sq{i}"]))
    exact.append(V("v_sub_co_u32 %[h0], %[sk0], %[a0], %[b0]", ["sk0"]))
    exact.append(V("v_subb_co_u32 %[h1], %[scy], %[a1], %[b1], %[sk0]", ["scy"], ["sk0"]))
    for i in (1, 2, 3):
        exact.append(V(f"v_subb_co_u32 %[h{2 * i}], %[sk0], %[a{2 * i}], %[b{2 * i}], %[scy]", ["sk0"], ["scy"]))
        exact.append(V(f"v_subb_co_u32 %[h{2 * i + 1}], %[sk1], %[a{2 * i + 1}], %[b{2 * i + 1}], %[sk0]",
                       ["sk1"], ["sk0"]))
        exact.append(S(f"s_and_b64 %[sq{i}], %[sq{i}], %[scy]", [f"sq{i}"]))
        exact.append(S(f"s_andn2_b64 %[scy], %[sk1], %[sq{i}]", ["scy"]))      # lossy borrow
    exactp = [V("v_cndmask_b32 %[vt1], 0, 19, %[scy]", [], ["scy"]),
              V("v_cndmask_b32 %[vt2], 0, %[c80], %[scy]", [], ["scy"]),
              V("v_sub_co_u32 %[h0], %[sk0], %[h0], %[vt1]", ["sk0"]),
              V("v_subb_co_u32 %[h1], %[sd1], %[h1], 0, %[sk0]", ["sd1"], ["sk0"]),        # d1 = m & t0 < 19
              V("v_subb_co_u32 %[h2], %[sk1], %[h2], 0, %[sd1]", ["sk1"], ["sd1"]),
              V("v_subb_co_u32 %[h3], %[sk1], %[h3], 0, %[sk1]", ["sk1"], ["sk1"]),
              V("v_and_b32 %[vt1], %[h2], %[h3]"),
              V("v_cmp_eq_u32 %[sd2], -1, %[vt1]", ["sd2"]),
              S("s_and_b64 %[sd2], %[sd2], %[scy]", ["sd2"]),                              # d2 = m & o1 == M
              V("v_subb_co_u32 %[h4], %[sk2], %[h4], 0, %[sd2]", ["sk2"], ["sd2"]),
              V("v_subb_co_u32 %[h5], %[sk2], %[h5], 0, %[sk2]", ["sk2"], ["sk2"]),
              V("v_and_b32 %[vt1], %[h4], %[h5]"),
              V("v_cmp_eq_u32 %[sd3], -1, %[vt1]", ["sd3"]),
              S("s_and_b64 %[sd3], %[sd3], %[scy]", ["sd3"]),                              # d3 = m & o2 == M
              V("v_subb_co_u32 %[h6], %[sk3], %[h6], 0, %[sd3]", ["sk3"], ["sd3"]),
              V("v_subb_co_u32 %[h7], %[sk3], %[h7], 0, %[sk3]", ["sk3"], ["sk3"]),
              V("v_add_u32 %[h7], %[h7], %[vt2]")]                                         # + m 2^63
    # fast statement: test 1's max of the g words first, the plain chain, test 2's words into the same
    # max and the one compare as soon as t1, t2 and t4 exist, the rest of the chain, the fast "+ p".
    # Exact statement (any rare lane): the exact chain from the inputs again and the exact "+ p"
    # (the exact chain equals the plain one when test 1 finds no lane, so this covers test 2 alone).
    fast = [V("v_max3_u32 %[vt3], %[b2], %[b4], %[b6]")] + plain[:5] + \
        [V("v_not_b32 %[vt1], %[h1]"),
         V("v_max3_u32 %[vt3], %[vt3], %[vt1], %[h2]"),
         V("v_max_u32 %[vt3], %[vt3], %[h4]"),
         V("v_cmp_eq_u32 %[srare], -1, %[vt3]", ["srare"])] + plain[5:] + fastp
    lf, _ = schedule(fast)
    ls, _ = schedule(exact + exactp)
    return emit_split("fe_sub_asm", ["fe25519_sub (curve25519_ops.cu:71-90) on limb halves: lossy borrow chain, then the",
                                     "literal \"+ p\" pass on a final borrow (fast forms unless a lane is on a rare edge)."],
                      [("fa", "a"), ("ga", "b")], t, ["vt1", "vt2", "vt3"], ["scy", "srare", "sk0"], lf,
                      ["sk0", "sk1", "sk2", "sk3", "sd1", "sd2", "sd3", "scy", "sq1", "sq2", "sq3"], ls)


def renamed(ins, names):
    """ins with its %[x] operands (and SGPR write/read lists) renamed by names {old: new}."""
    out = []
    for text, w, r, v in ins:
        for a, b in names.items():
            text = text.replace(f"%[{a}]", f"%[{b}]")
        out.append((text, [names.get(x, x) for x in w], [names.get(x, x) for x in r], v))
    return out


def gen_addsub(lat=False, acc=False):
    """fe_add(a, b) and fe_sub(a, b) of the same operands in one block (ge25519_add's E = B - A with
    H = B + A, and F = D - C with G = D + C; the lane-quad forms' next operands Y - X / Y + X), for
    the latency-bound drain chains: the two carry chains interleaved, so a link reads its carry two
    instructions after the write (an s_nop 0 instead of an s_nop 1 per link), and one wave-uniform
    rare-edge branch for both: sub's test 1 (some g_i, i = 1..3, may be 2^64-1), add's fix_test and
    sub's test 2, OR-ed.  Fast path: add's fast fix-up and sub's fast "+ p".  Slow path: both from
    the inputs again, exactly as fe_add_asm and fe_sub_asm do (add chain + fix_seq; sub's exact chain
    + exact "+ p").  Same bits as the two separate blocks."""
    h = [f"h{i}" for i in range(8)]   # a + b
    chains = [V("v_add_co_u32 %[h0], %[scy], %[a0], %[b0]", ["scy"]),
              V("v_sub_co_u32 %[t0], %[sby], %[a0], %[b0]", ["sby"])]
    for i in range(1, 8):
        chains.append(V(f"v_addc_co_u32 %[h{i}], %[scy], %[a{i}], %[b{i}], %[scy]", ["scy"], ["scy"]))
        chains.append(V(f"v_subb_co_u32 %[t{i}], %[sby], %[a{i}], %[b{i}], %[sby]", ["sby"], ["sby"]))
    # one max over every word the three tests read (sub's test 1: g words; add's fix_test: h1, h4;
    # sub's test 2: ~t1, t2, t4), compared as soon as the chains have produced limb 4's words
    pre = [V("v_max3_u32 %[vt3], %[b2], %[b4], %[b6]")] + chains[:10] + \
        [V("v_not_b32 %[vt4], %[t1]"),
         V("v_max3_u32 %[vt3], %[vt3], %[h1], %[h4]"),
         V("v_max3_u32 %[vt3], %[vt3], %[vt4], %[t2]"),
         V("v_max_u32 %[vt3], %[vt3], %[t4]"),
         V("v_cmp_eq_u32 %[srare], -1, %[vt3]", ["srare"])] + chains[10:]
    if not lat:
        pre += [V("v_cmp_gt_i32 %[stp], 0, %[h7]", ["stp"]), S("s_or_b64 %[sm], %[scy], %[stp]", ["sm"])]
    fast = [V("v_cndmask_b32 %[vt1], 0, 19, %[sm]", [], ["sm"]),
            V("v_cndmask_b32 %[vt4], 0, 19, %[sby]", [], ["sby"]),
            V("v_cndmask_b32 %[vt2], 0, %[c80], %[sm]", [], ["sm"]),
            V("v_cndmask_b32 %[vt5], 0, %[c80], %[sby]", [], ["sby"]),
            V("v_add_co_u32 %[h0], %[sk0], %[h0], %[vt1]", ["sk0"]),
            V("v_sub_co_u32 %[t0], %[sk1], %[t0], %[vt4]", ["sk1"]),
            V("v_addc_co_u32 %[h4], %[sk2], %[h4], 0, %[sm]", ["sk2"], ["sm"]),
            V("v_add_u32 %[h7], %[h7], %[vt2]"),
            V("v_add_u32 %[t7], %[t7], %[vt5]"),
            V("v_addc_co_u32 %[h1], %[sk0], %[h1], 0, %[sk0]", ["sk0"], ["sk0"]),
            V("v_subb_co_u32 %[t1], %[sk1], %[t1], 0, %[sk1]", ["sk1"], ["sk1"]),
            V("v_addc_co_u32 %[h5], %[sk2], %[h5], 0, %[sk2]", ["sk2"], ["sk2"])]
    if lat:   # add's m = carry | top as a VALU mask (fix_fast_lat), sub's "+ p" as above, interleaved
        fast = [V("v_ashrrev_i32 %[vt2], 31, %[h7]"),
                V("v_cndmask_b32 %[vt4], 0, 19, %[sby]", [], ["sby"]),
                V("v_cndmask_b32 %[vt2], %[vt2], -1, %[scy]", [], ["scy"]),
                V("v_cndmask_b32 %[vt5], 0, %[c80], %[sby]", [], ["sby"]),
                V("v_and_b32 %[vt1], 19, %[vt2]"),
                V("v_lshrrev_b32 %[vt3], 31, %[vt2]"),
                V("v_and_b32 %[vt2], %[c80], %[vt2]"),
                V("v_add_co_u32 %[h0], %[sk0], %[h0], %[vt1]", ["sk0"]),
                V("v_sub_co_u32 %[t0], %[sk1], %[t0], %[vt4]", ["sk1"]),
                V("v_add_co_u32 %[h4], %[sk2], %[h4], %[vt3]", ["sk2"]),
                V("v_add_u32 %[h7], %[h7], %[vt2]"),
                V("v_add_u32 %[t7], %[t7], %[vt5]"),
                V("v_addc_co_u32 %[h1], %[sk0], %[h1], 0, %[sk0]", ["sk0"], ["sk0"]),
                V("v_subb_co_u32 %[t1], %[sk1], %[t1], 0, %[sk1]", ["sk1"], ["sk1"]),
                V("v_addc_co_u32 %[h5], %[sk2], %[h5], 0, %[sk2]", ["sk2"], ["sk2"])]
    add_exact = [V("v_add_co_u32 %[h0], %[scy], %[a0], %[b0]", ["scy"])]
    for i in range(1, 8):
        add_exact.append(V(f"v_addc_co_u32 %[h{i}], %[scy], %[a{i}], %[b{i}], %[scy]", ["scy"], ["scy"]))
    add_exact += fix_seq(h, h, "scy")
    # sub's exact chain + exact "+ p" (gen_sub's sequences) on t, its borrow in sby
    sub_exact = []
    for i in (1, 2, 3):
        sub_exact.append(V(f"v_and_b32 %[vt1], %[b{2 * i}], %[b{2 * i + 1}]"))
        sub_exact.append(V(f"v_cmp_eq_u32 %[sq{i}], -1, %[vt1]", [f"sq{i}"]))
    sub_exact.append(V("v_sub_co_u32 %[t0], %[sk0], %[a0], %[b0]", ["sk0"]))
    sub_exact.append(V("v_subb_co_u32 %[t1], %[sby], %[a1], %[b1], %[sk0]", ["sby"], ["sk0"]))
    for i in (1, 2, 3):
        sub_exact.append(V(f"v_subb_co_u32 %[t{2 * i}], %[sk0], %[a{2 * i}], %[b{2 * i}], %[sby]", ["sk0"], ["sby"]))
        sub_exact.append(V(f"v_subb_co_u32 %[t{2 * i + 1}], %[sk1], %[a{2 * i + 1}], %[b{2 * i + 1}], %[sk0]",
                           ["sk1"], ["sk0"]))
        sub_exact.append(S(f"s_and_b64 %[sq{i}], %[sq{i}], %[sby]", [f"sq{i}"]))
        sub_exact.append(S(f"s_andn2_b64 %[sby], %[sk1], %[sq{i}]", ["sby"]))
    sub_exact += renamed([
        V("v_cndmask_b32 %[vt1], 0, 19, %[scy]", [], ["scy"]),
        V("v_cndmask_b32 %[vt2], 0, %[c80], %[scy]", [], ["scy"]),
        V("v_sub_co_u32 %[h0], %[sk0], %[h0], %[vt1]", ["sk0"]),
        V("v_subb_co_u32 %[h1], %[sd1], %[h1], 0, %[sk0]", ["sd1"], ["sk0"]),
        V("v_subb_co_u32 %[h2], %[sk1], %[h2], 0, %[sd1]", ["sk1"], ["sd1"]),
        V("v_subb_co_u32 %[h3], %[sk1], %[h3], 0, %[sk1]", ["sk1"], ["sk1"]),
        V("v_and_b32 %[vt1], %[h2], %[h3]"),
        V("v_cmp_eq_u32 %[sd2], -1, %[vt1]", ["sd2"]),
        S("s_and_b64 %[sd2], %[sd2], %[scy]", ["sd2"]),
        V("v_subb_co_u32 %[h4], %[sk2], %[h4], 0, %[sd2]", ["sk2"], ["sd2"]),
        V("v_subb_co_u32 %[h5], %[sk2], %[h5], 0, %[sk2]", ["sk2"], ["sk2"]),
        V("v_and_b32 %[vt1], %[h4], %[h5]"),
        V("v_cmp_eq_u32 %[sd3], -1, %[vt1]", ["sd3"]),
        S("s_and_b64 %[sd3], %[sd3], %[scy]", ["sd3"]),
        V("v_subb_co_u32 %[h6], %[sk3], %[h6], 0, %[sd3]", ["sk3"], ["sd3"]),
        V("v_subb_co_u32 %[h7], %[sk3], %[h7], 0, %[sk3]", ["sk3"], ["sk3"]),
        V("v_add_u32 %[h7], %[h7], %[vt2]")], {**{f"h{i}": f"t{i}" for i in range(8)}, "scy": "sby"})
    lf, _ = schedule(pre + fast)
    if acc:
        return emit_acc("fe_addsub_asm_lat_acc", ["fe_addsub_asm_lat's fast statement, the rare-edge test deferred into acc (emit_acc)."],
                        [("fa", "a"), ("ga", "b")], h + [f"t{i}" for i in range(8)],
                        ["vt1", "vt2", "vt3", "vt4", "vt5"], ["scy", "sby", "sk0", "sk1", "sk2"],
                        schedule(to_acc(pre + fast))[0])
    ls, _ = schedule(add_exact + sub_exact)
    return emit_split("fe_addsub_asm" + ("_lat" if lat else ""), ["fe_add(a, b) and fe_sub(a, b) in one block (curve25519_ops.cu:41-90): the two carry",
                                        "chains interleaved, one rare-edge test for both (tools/gen_field_asm.py gen_addsub)."],
                      [("fa", "a"), ("ga", "b")], h + [f"t{i}" for i in range(8)], ["vt1", "vt2", "vt3", "vt4", "vt5"],
                      ["scy", "sby", "srare", "sk0", "sk1", "sk2"] + ([] if lat else ["stp", "sm"]), lf,
                      FIX_SGPRS + ["scy", "sby", "sq1", "sq2", "sq3"], ls)


def gen_canon():
    """host fe25519_tobytes' conditional "- p" (curve25519_ops.cu:220-251) = device fe_mul_one:
    the fix-up with no carry, in place."""
    h = [f"h{i}" for i in range(8)]
    lines = two_way(fix_test(h, "0"), fix_fast(h), fix_seq(h, h, "0"))
    return emit("fe_canon_asm", ["Canonicalising \"- p\" of fe25519_tobytes (curve25519_ops.cu:220-251), in place:",
                                 "h >= p ? lossy - p : h (fast form unless a lane is on a rare edge)."],
                [("ha", "h")], [], h, ["vt1", "vt2", "vt3"], FIX_SGPRS + ["srare"], lines, inout=True)


def gen_q4_sum():
    """The lane quad's two DPP levels of fe_q4_sum_fold (ge25519_quad.h) as one scheduled block:
    level 1 (quad_perm [1,1,3,3]) q = w + (lane|1's w) << 64 bits on lanes 0 and 2, level 2 (quad_perm
    [2,2,2,2]) r = q + (lane 2's q) << 128 bits on lane 0 -- the exact 512-bit sum of the four 320-bit
    partials.  The two carry chains (SGPR pairs sa, sb) and the 22 DPP moves are list-scheduled
    together so each link finds its carry 1 wait state after the write and each DPP its source 2
    after (the compiler left one wait per link of both chains: 57 of a row step's wait states)."""
    ins = []   # (name, text, deps [(name, min distance in slots)], writes)
    for k in range(10):
        ins.append((f"d1_{k}", f"v_mov_b32_dpp %[n{k}], %[w{k}] quad_perm:[1,1,3,3] row_mask:0xf bank_mask:0xf "
                    "bound_ctrl:1", []))
    qsrc = lambda j: None if j < 2 else f"l1_{j}"
    for i in range(2, 12):
        a = f"%[w{i}]" if i < 10 else "0"
        b = f"%[n{i - 2}]"
        deps = [(f"d1_{i - 2}", 1)] + ([(f"l1_{i - 1}", 2)] if i > 2 else [])
        if i == 2:
            ins.append((f"l1_{i}", f"v_add_co_u32 %[q{i}], %[sa], {a}, {b}", deps))
        else:
            ins.append((f"l1_{i}", f"v_addc_co_u32 %[q{i}], %[sa], {a}, {b}, %[sa]", deps))
    for j in range(12):
        src = f"%[w{j}]" if j < 2 else f"%[q{j}]"
        deps = [] if j < 2 else [(f"l1_{j}", 3)]   # a VALU-written VGPR read by DPP: 2 wait states
        ins.append((f"d2_{j}", f"v_mov_b32_dpp %[m{j}], {src} quad_perm:[2,2,2,2] row_mask:0xf bank_mask:0xf "
                    "bound_ctrl:1", deps))
    for i in range(4, 16):
        a = f"%[q{i}]" if i < 12 else "0"
        deps = [(f"d2_{i - 4}", 1)] + ([(f"l1_{i}", 1)] if i < 12 else []) + ([(f"l2_{i - 1}", 2)] if i > 4 else [])
        if i == 4:
            ins.append((f"l2_{i}", f"v_add_co_u32 %[r{i}], %[sb], {a}, %[m{i - 4}]", deps))
        else:
            ins.append((f"l2_{i}", f"v_addc_co_u32 %[r{i}], %[sb], {a}, %[m{i - 4}], %[sb]", deps))
    # list scheduling: each slot takes the first ready instruction, chains first (longest remaining
    # path), else a wait state
    prio = {n: (0 if n.startswith("l2") else 1 if n.startswith("l1") else 2 if n.startswith("d2") else 3)
            for n, _, _ in ins}
    pos, lines, t = {}, ["s_nop 1"], 0   # the w words may have been written just before the block
    left = list(ins)
    while left:
        ready = [x for x in left if all(d in pos and t >= pos[d] + dist for d, dist in x[2])]
        if not ready:
            lines.append("s_nop 0")
            t += 1
            continue
        x = min(ready, key=lambda x: (prio[x[0]], left.index(x)))
        lines.append(x[1])
        pos[x[0]] = t
        left.remove(x)
        t += 1
    outs = [f"q{i}" for i in range(2, 12)] + [f"r{i}" for i in range(4, 16)] + [f"n{k}" for k in range(10)] + \
           [f"m{j}" for j in range(12)]
    text = "\\n\\t".join(lines)
    out = ["// fe_q4_sum_fold's two DPP levels (ge25519_quad.h) in one list-scheduled block: r[0..15] (valid on",
           f"// the quad's lane 0) = the sum of the quad's four partials w[0..9] at word offsets 0, 2, 4, 6 ({t} slots).",
           "__device__ __forceinline__ void q4_sum_asm(uint32_t r[16], const uint32_t w[10]) {",
           "    const uint32_t " + ", ".join(f"w{k} = w[{k}]" for k in range(10)) + ";",
           "    uint32_t " + ", ".join(outs) + ";",
           "    uint64_t sa, sb;",
           f'    asm volatile("{text}"',
           "                 : " + ", ".join([f'[{x}] "=&v"({x})' for x in outs] + ['[sa] "=&s"(sa)', '[sb] "=&s"(sb)']),
           "                 : " + ", ".join(f'[w{k}] "v"(w{k})' for k in range(10)) + ");",
           "    r[0] = w0; r[1] = w1; r[2] = q2; r[3] = q3;",
           "    " + " ".join(f"r[{i}] = r{i};" for i in range(4, 16)),
           "    (void)sa; (void)sb; " + " ".join(f"(void){x};" for x in [f"q{i}" for i in range(12, 12)]),
           "}"]
    return out


def main(path=OUT):
    out = ["// GENERATED by tools/gen_field_asm.py -- do not edit by hand.",
           "// gfx950 inline-asm fe25519 add and product fold: the same bits as the C forms in fe25519_dev.h.",
           "#pragma once", "#include <stdint.h>", "namespace bp {"]
    out += gen_add() + [""] + gen_sub() + [""] + gen_fold() + [""] + gen_canon() + [""] + gen_addsub() + [""] + \
        gen_q4_sum() + [""]
    out += ["// Latency forms (the 16-lane row step, one wave per SIMD): the same blocks with m = carry | top",
            "// computed in VALU (fix_fast_lat) instead of a compare + SALU OR; same bits."]
    out += gen_add(lat=True) + [""] + gen_fold(lat=True) + [""] + gen_addsub(lat=True) + [""]
    out += ["// The row step's fast statements with the rare-edge test deferred (emit_acc; ge25519_quad.h sm_row)."]
    out += gen_add(lat=True, acc=True) + [""] + gen_fold(lat=True, acc=True) + [""] + gen_addsub(lat=True, acc=True)
    out.append("}  // namespace bp")
    open(path, "w").write("\n".join(out) + "\n")
    print("wrote", path)


if __name__ == "__main__":
    main()
