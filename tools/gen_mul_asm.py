"""Generate cudabulletproof_amd/csrc/mul512_asm.h: the exact 256x256 -> 512-bit product as
product-scanning columns of gfx950 `v_mad_u64_u32` (64-bit accumulate, carry-out to an SGPR
lane mask) + `v_addc_co_u32` (carry count), one asm statement per column.

Hazard rule applied inside each statement: a VALU write of an SGPR lane mask is read by a
VALU carry-in no sooner than 1 wait state later (intervening VALU instructions count 1 each,
`s_nop N` counts N+1): the spacing the compiler gives its own e64 carry chains on gfx950
(tools/hazard_probe.hip read no stale carry even at 0 on MI355X; rounds 1-6 used 2).
"""
import os

HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(HERE, "..", "cudabulletproof_amd", "csrc", "mul512_asm.h")
WAIT = 1


def column(k, square=False):
    prods = [(i, k - i) for i in range(8) if 0 <= k - i <= 7]
    return prods


def offdiag(k):
    """Products a_i a_j, i < j, of column k (the squaring's off-diagonal half)."""
    return [(i, k - i) for i in range(8) if i < k - i <= 7]


def emit_column(k, prods=None, first=None, bounded=False):
    """One product-scanning column as asm lines.  bounded (an int, True = 1): that many leading
    products of the column cannot carry out of the 64-bit accumulator (the caller has checked the
    operand words that bound them, see BOUNDED below), so only the later products' carries are
    counted.  Returns (prods, lines, counted) with counted = the number of carries counted into c2
    (0: c2 is not written)."""
    prods = column(k) if prods is None else prods
    first = (k == 0) if first is None else first
    need_carry = not first
    pending = []      # sgpr indices whose carry is still to be counted
    seq = []
    counted = 0
    for t, (i, j) in enumerate(prods):
        s = t % 3
        skip = need_carry and t < int(bounded)
        seq.append(("mad", i, j, "sd" if skip else f"s{s}", t))
        if need_carry and not skip:
            pending.append(s)
            counted += 1
        if len(pending) > 2:
            seq.append(("addc", pending.pop(0)))
    while need_carry and pending:
        seq.append(("addc", pending.pop(0)))
    # lay out with nops
    lines, pos, wpos = [], 0, {}
    first_addc = True
    for op in seq:
        if op[0] == "mad":
            _, i, j, sname, t = op
            if first and t == 0:
                lines.append(f"v_mad_u64_u32 %[acc], %[{sname}], %[a{i}], %[b{j}], 0")
            else:
                lines.append(f"v_mad_u64_u32 %[acc], %[{sname}], %[a{i}], %[b{j}], %[acc]")
            if sname != "sd":
                wpos[int(sname[1:])] = pos
            pos += 1
        else:
            s = op[1]
            gap = pos - wpos[s] - 1
            if gap < WAIT:
                lines.append(f"s_nop {WAIT - gap - 1}")
                pos += WAIT - gap
            if first_addc:   # c2 = carry (no separate zeroing)
                lines.append(f"v_addc_co_u32 %[c2], %[sd], 0, 0, %[s{s}]")
                first_addc = False
            else:
                lines.append(f"v_addc_co_u32 %[c2], %[sd], %[c2], 0, %[s{s}]")
            pos += 1
    return prods, lines, counted


# The bounded forms.  Column k's FIRST product is a_0 b_k (k <= 7) or a_(k-7) b_7 (k >= 8) (column()
# and offdiag() list products in increasing i), and it is added to the previous column's carry-out
# acc_start = hi + 2^32 c2 <= (2^32 - 1) + 2^32 (products of that column - 1) <= 2^35 - 1.  When the
# gating words a_0 and b_7 (a_0 and a_7 for a square) are <= 0xFFFFFFEF, that product is at most
# (2^32 - 1)(2^32 - 17) = 2^64 - 18 2^32 + 17, so acc_start + it < 2^64 - 10 2^32 + 17: no carry
# out, and the column need not count it.  mul512 / sqr512 test the gating words wave-uniformly and
# run the counting form when any lane exceeds the bound (probability ~2^-27 per lane).
BOUNDED = 0xFFFFFFEF


# Multiplication by the curve constant k (= d, curve25519_ops.cu:341-346; the C of every point
# operation, C = (T1 T2) k).  Seven of d's eight 32-bit words are below 2^31, so a column's products
# by them can be summed further before the 64-bit accumulator can overflow.  Each column takes its
# products smallest word first; with every word of the variable operand at most 2^32 - 1, a bound of
# the column's true running sum (the carry-in bound of the column before + the products so far)
# decides which products could carry out: only those are counted (16 of 64; the bounded general
# product counts 50).  The words are wave-uniform, so they are SGPR operands.
K_CONST = (0x75EB4DCA135978A3, 0x00700A4D4141D8AB, 0x8CC740797779E898, 0x52036CEE2B6FFE73)


def k_words():
    w = []
    for limb in K_CONST:
        w += [limb & 0xFFFFFFFF, limb >> 32]
    return w


def k_columns(rows=8):
    """[(k, prods ordered smallest word first, first, uncounted)] and the total counted carries, for
    the product of `rows` words of a (8: the whole product; 2: a lane's two rows of fe_mul_q4) by k."""
    kw = k_words()
    M = 2**32 - 1
    cin, cols, total = 0, [], 0
    for k in range(rows + 7):
        prods = sorted(((i, k - i) for i in range(rows) if 0 <= k - i <= 7), key=lambda ij: kw[ij[1]])
        bound, counted = cin, 0
        for _, j in prods:
            if bound + M * kw[j] >= 2**64:
                counted += 1
            bound += M * kw[j]
        cols.append((k, prods, k == 0, len(prods) - counted))
        total += counted
        cin = bound >> 32
    return cols, total


def emit_product(out, fname, sig, wname, cols, last, bounded=False, square=False, pre=(), uncounted=None,
                 bconst=None):
    """One generated product function.  cols = [(k, prods, first)]: column k's words go to
    wname[k]; `last` = the index of the final carry word (wname[last] = the accumulator's high part).
    square: operand b is a (the off-diagonal half of a square)."""
    out.append(f"__device__ __forceinline__ void {fname}({sig}) {{")
    out.append("    uint64_t acc = 0, s0, s1, s2, sd;")
    out.append("    uint32_t c2;")
    out.extend(pre)
    prev_counted = 0
    for idx, (k, prods, first) in enumerate(cols):
        _, lines, counted = emit_column(k, prods, first=first, bounded=uncounted(k) if uncounted else bounded)
        if idx > 0:   # the previous column's carry-out: (acc >> 32) + 2^32 (its counted carries)
            out.append("    acc = (acc >> 32) | ((uint64_t)c2 << 32);" if prev_counted else "    acc >>= 32;")
        ai = sorted({i for i, _ in prods} | ({j for _, j in prods} if square else set()))
        bj = [] if square else sorted({j for _, j in prods})
        body = "\\n\\t".join(lines)
        if square:
            body = body.replace("%[b", "%[a")
        bop = (lambda j: f'[b{j}] "s"({bconst}[{j}])') if bconst else (lambda j: f'[b{j}] "v"(b[{j}])')
        ops_in = ", ".join([f'[a{i}] "v"(a[{i}])' for i in ai] + [bop(j) for j in bj])
        if first:
            out.append(f'    asm volatile("{body}" : [acc] "=&v"(acc), [s0] "=&s"(s0) : {ops_in});')
        elif counted:
            out.append(f'    asm volatile("{body}"')
            out.append(f'                 : [acc] "+v"(acc), [c2] "=&v"(c2), [s0] "=&s"(s0), [s1] "=&s"(s1), '
                       f'[s2] "=&s"(s2), [sd] "=&s"(sd)')
            out.append(f"                 : {ops_in});")
        else:
            out.append(f'    asm volatile("{body}"')
            out.append(f'                 : [acc] "+v"(acc), [s0] "=&s"(s0), [s1] "=&s"(s1), [s2] "=&s"(s2), '
                       f'[sd] "=&s"(sd)')
            out.append(f"                 : {ops_in});")
        out.append(f"    {wname}[{k}] = (uint32_t)acc;")
        prev_counted = counted
    out.append("    acc = (acc >> 32) | ((uint64_t)c2 << 32);" if prev_counted else "    acc >>= 32;")
    out.append(f"    {wname}[{last}] = (uint32_t)acc;")
    if square:
        out.append(f"    {wname}[{last + 1}] = (uint32_t)(acc >> 32);")
    out.append("    (void)s0; (void)s1; (void)s2; (void)sd; (void)c2;")
    out.append("}")
    out.append("")


def main(path=OUT):
    out = []
    out.append("// GENERATED by tools/gen_mul_asm.py -- do not edit by hand.")
    out.append("// Exact 256x256 -> 512-bit product, product scanning, one asm statement per column.")
    out.append("#pragma once")
    out.append("#include <stdint.h>")
    out.append("namespace bp {")
    out.append(f"// Gating-word bound of the *_bounded forms (tools/gen_mul_asm.py BOUNDED): every column's first")
    out.append(f"// product is known not to carry out when the gating words are <= it, so it is not counted.")
    out.append(f"constexpr uint32_t MUL_BOUNDED_WORD = 0x{BOUNDED:08X}u;")
    full = [(k, column(k), k == 0) for k in range(15)]
    for bounded, suffix in ((False, ""), (True, "_bounded")):
        if bounded:
            out.append("// The same product with the first carry of every column uncounted: valid when a[0] and b[7]")
            out.append("// are <= MUL_BOUNDED_WORD (14 carry counts fewer).")
        emit_product(out, f"mul512{suffix}_asm", "uint32_t w[16], const uint32_t a[8], const uint32_t b[8]", "w", full,
                     15, bounded=bounded)
    off = [(k, offdiag(k), k == 1) for k in range(1, 14)]
    for bounded, suffix in ((False, ""), (True, "_bounded")):
        out.append("// Off-diagonal half of a square: o = sum_{i<j} a_i a_j 2^(32(i+j)), o[0] = 0 (columns 1..13)"
                   + (";" if bounded else "."))
        if bounded:
            out.append("// bounded: the first carry of every column uncounted, valid when a[0], a[7] <= MUL_BOUNDED_WORD.")
        emit_product(out, f"sqr512_offdiag{suffix}_asm", "uint32_t o[16], const uint32_t a[8]", "o", off, 14,
                     bounded=bounded, square=True, pre=("    o[0] = 0;",))
    out.append("// Two rows of the product for a lane quad that shares one multiplication: (a1 2^32 + a0) * b,")
    out.append("// the exact 320-bit partial as 10 words (columns 0..8 + the final carry word).")
    # column 8's single product a_1 b_7 never carries out in either form: the partial is < 2^320
    rows2 = [(k, [(i, k - i) for i in range(2) if 0 <= k - i <= 7], k == 0) for k in range(9)]
    emit_product(out, "mul2x8_asm", "uint32_t w[10], const uint32_t a[2], const uint32_t b[8]", "w", rows2, 9,
                 uncounted=lambda k: 1 if k == 8 else 0)
    out.append("// bounded: each column's first product a_0 b_k uncounted (columns 1..7 keep one count), valid when")
    out.append("// a[0] <= MUL_BOUNDED_WORD (acc_start <= 2^33 - 1 here: at most one counted carry per column).")
    emit_product(out, "mul2x8_bounded_asm", "uint32_t w[10], const uint32_t a[2], const uint32_t b[8]", "w", rows2,
                 9, uncounted=lambda k: 1)
    kcols, kcount = k_columns()
    out.append(f"// a * k (k = d, the curve constant of every point addition): the exact 512-bit product with only")
    out.append(f"// the carries a column's running-sum bound allows counted ({kcount} of 64); valid for any a.")
    kw = ", ".join(f"0x{w:08X}u" for w in k_words())
    unc = {k: u for k, _, _, u in kcols}
    emit_product(out, "mul512_k_asm", "uint32_t w[16], const uint32_t a[8]", "w",
                 [(k, prods, first) for k, prods, first, _ in kcols], 15, uncounted=lambda k: unc[k],
                 bconst="kw", pre=(f"    constexpr uint32_t kw[8] = {{{kw}}};",))
    kcols2, kcount2 = k_columns(2)
    out.append(f"// A lane's two rows of fe_mul_q4(x, k): (a1 2^32 + a0) * k as 10 words, {kcount2} carries counted (the")
    out.append(f"// bounded general rows count 7).")
    unc2 = {k: u for k, _, _, u in kcols2}
    emit_product(out, "mul2x8_k_asm", "uint32_t w[10], const uint32_t a[2]", "w",
                 [(k, prods, first) for k, prods, first, _ in kcols2], 9, uncounted=lambda k: unc2[k],
                 bconst="kw", pre=(f"    constexpr uint32_t kw[8] = {{{kw}}};",))
    out.append("}  // namespace bp")
    open(path, "w").write("\n".join(out) + "\n")
    print("wrote", path)


if __name__ == "__main__":
    main()
