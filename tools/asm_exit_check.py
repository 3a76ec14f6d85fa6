"""Scan every compiled kernel of the library for a memory instruction (VMEM or SMEM) that reads an
SGPR written by a VALU instruction inside an inline-asm block fewer than 5 wait states earlier (the
gfx9 "VALU writes SGPR -> VMEM reads it" hazard), following fall-through and branch targets from
each block's end.  The generated field blocks (tools/gen_field_asm.py) end without a guard, so this
must print "flags 0".

  python tools/asm_exit_check.py
"""
import re, subprocess, sys, glob, os, tempfile
tmp = tempfile.mkdtemp()
SRC = sorted(glob.glob(os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', 'cudabulletproof_amd', 'csrc', '*.hip')))
def regs(tok):
    tok = tok.strip().rstrip(',')
    m = re.match(r's\[(\d+):(\d+)\]$', tok)
    if m: return {f's{i}' for i in range(int(m.group(1)), int(m.group(2)) + 1)}
    m = re.match(r's(\d+)$', tok)
    if m: return {tok}
    if tok in ('vcc',): return {'vcc_lo', 'vcc_hi'}
    if tok in ('vcc_lo', 'vcc_hi'): return {tok}
    return set()
def ops(line):
    parts = line.split(None, 1)
    if len(parts) < 2: return parts[0], []
    return parts[0], [p.strip() for p in parts[1].split(',')]
VALU_SDST2 = ('v_add_co_u32', 'v_addc_co_u32', 'v_sub_co_u32', 'v_subb_co_u32', 'v_subrev_co_u32', 'v_subbrev_co_u32',
              'v_mad_u64_u32', 'v_mad_i64_i32', 'v_div_scale')
flags = 0; blocks = 0
def compile_one(src):
    out = os.path.join(tmp, os.path.basename(src) + '.s')
    subprocess.run(['hipcc', '--offload-arch=gfx950', '-O3', '-std=c++17', '-S', '--cuda-device-only', src, '-o', out],
                   check=True, stderr=subprocess.DEVNULL)
    return out
from concurrent.futures import ThreadPoolExecutor
with ThreadPoolExecutor(max_workers=min(8, os.cpu_count() or 1)) as pool:
    outs = list(pool.map(compile_one, SRC))
for src, out in zip(SRC, outs):
    lines = [l.strip() for l in open(out)]
    i = 0
    while i < len(lines):
        if lines[i].startswith(';;#ASMSTART'):
            j = i + 1; written = {}
            pos = 0
            while not lines[j].startswith(';;#ASMEND'):
                t = lines[j]
                if t and not t.startswith(';') and not t.endswith(':'):
                    op, a = ops(t)
                    base = op.split('_e32')[0].split('_e64')[0]
                    if op.startswith('v_'):
                        if base in VALU_SDST2 and len(a) > 1 and not op.endswith('_e32'):
                            for r in regs(a[1]): written[r] = pos
                        elif base.startswith('v_cmp') and a and not op.endswith('_e32'):
                            for r in regs(a[0]): written[r] = pos
                        elif op.endswith('_e32') and (base in VALU_SDST2 or base.startswith('v_cmp')):
                            written['vcc_lo'] = written['vcc_hi'] = pos
                    elif op.startswith('s_') and a:
                        if op.startswith('s_nop'):
                            pos += int(a[0]) if a else 0
                        elif not op.startswith(('s_cmp', 's_cbranch', 's_branch', 's_waitcnt')):
                            for r in regs(a[0]): written.pop(r, None)   # a SALU write replaces it
                    pos += 1
                j += 1
            blocks += 1
            end = pos
            live = {r: end - p - 1 for r, p in written.items()}   # wait states since the write at block end
            # scan forward along every path (fall-through and branch targets) for 6 wait states
            labels = {}
            def label_index(name):
                if name not in labels:
                    for q in range(len(lines)):
                        if lines[q] == name + ':' or lines[q].startswith(name + ':'):
                            labels[name] = q
                            break
                return labels.get(name)
            stack = [(j + 1, 0, dict(live))]
            seen = set()
            while stack:
                k, dist, lv = stack.pop()
                while k < len(lines) and dist < 6 and lv:
                    if (k, dist) in seen:
                        break
                    seen.add((k, dist))
                    t = lines[k]
                    if t.startswith(';;#ASMSTART') or t.startswith('s_endpgm') or t.startswith('.Lfunc_end'):
                        break
                    if t and not t.startswith(';') and not t.startswith('.') and not t.endswith(':') and ':' not in t.split()[0]:
                        op, a = ops(t)
                        is_mem = op.startswith(('global_', 'buffer_', 'flat_', 'scratch_', 's_load', 's_buffer_load', 's_store', 's_dcache'))
                        if is_mem:
                            reads = a[1:] if op.startswith(('s_load', 's_buffer_load')) else a   # (an SMEM load's first operand is its destination)
                            for tok in reads:
                                for r in regs(tok):
                                    if r in lv and lv[r] + dist < 5:
                                        print(f'{os.path.basename(src)}:{k}: {t}   <- {r} VALU-written {lv[r] + dist} states before')
                                        flags += 1
                        if op in ('s_branch', 's_cbranch_scc0', 's_cbranch_scc1', 's_cbranch_vccz', 's_cbranch_vccnz',
                                  's_cbranch_execz', 's_cbranch_execnz'):
                            tgt = label_index(a[0]) if a else None
                            if tgt is not None:
                                stack.append((tgt + 1, dist + 1, dict(lv)))
                            if op == 's_branch':
                                break
                        if op.startswith('s_') and a and not op.startswith(('s_nop', 's_cmp', 's_cbranch', 's_branch', 's_waitcnt', 's_store', 's_dcache', 's_load', 's_buffer_load')):
                            for r in regs(a[0]): lv.pop(r, None)
                        if op.startswith('v_') and a:
                            for r in regs(a[0]): lv.pop(r, None)
                        dist += (int(a[0]) + 1) if op == 's_nop' else 1
                    k += 1
            i = j
        i += 1
print('asm blocks', blocks, 'flags', flags)
sys.exit(1 if flags else 0)
