#!/usr/bin/env python3
"""Static instruction mix per ;MARK phase of one kernel in a TGMS_MARKS assembly dump.
usage: isa_phases.py k.s kernel_symbol_substring"""
import re, sys, collections
src, sym = sys.argv[1], sys.argv[2]
lines, on = [], False
for l in open(src):
    if not on and l.startswith(sym) and ':' in l.split(';')[0]:
        on = True
    elif on:
        lines.append(l)
        if 's_endpgm' in l:
            break
phase = 'prologue'
cnt = collections.defaultdict(collections.Counter)
for l in lines:
    m = re.search(r';MARK (\w+)', l)
    if m:
        phase = m.group(1); continue
    t = l.strip().split()
    if not t or t[0].startswith(';') or t[0].startswith('.') or t[0].endswith(':'):
        continue
    op = t[0]
    if op.startswith('v_'):
        cat = 'f64' if '_f64' in op else ('cndmask' if 'cndmask' in op else ('accvgpr' if 'accvgpr' in op else ('mov' if 'mov' in op else 'int')))
        cnt[phase]['VALU'] += 1; cnt[phase][cat] += 1
    elif op.startswith('ds_'): cnt[phase]['LDS'] += 1
    elif op.startswith(('global_', 'buffer_')): cnt[phase]['VMEM'] += 1
    elif op.startswith('s_'): cnt[phase]['SALU'] += 1
for p, c in cnt.items():
    print(f"{p:14s} " + " ".join(f"{k}={v}" for k, v in sorted(c.items())))
