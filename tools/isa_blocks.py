#!/usr/bin/env python3
"""Diagnostic: per-basic-block view of one kernel in a `hipcc -S -gline-tables-only` listing.

For every block: its label, loop depth / header (from the compiler's comments), instruction counts
(VALU / SALU / v_mov / LDS / VMEM) and the source lines (`.loc` of the given file) it contains, so
copy-heavy blocks (phi copies of the register state) can be traced back to the code that made them.

    tools/isa_blocks.py k9g.s reg_apply_kernelILi9 [--file mt_apply_reg.hip] [--min-mov 8]
"""
import argparse
import re

ap = argparse.ArgumentParser()
ap.add_argument('asm')
ap.add_argument('kernel')
ap.add_argument('--file', default='mt_apply_reg.hip')
ap.add_argument('--min-mov', type=int, default=8)
ap.add_argument('--all', action='store_true')
a = ap.parse_args()

src = open(a.asm).read()
files = {m.group(1): m.group(2) for m in re.finditer(r'^\s*\.file\s+(\d+)\s+"[^"]*"\s+"([^"]+)"', src, re.M)}
files.update({m.group(1): m.group(2) for m in re.finditer(r'^\s*\.file\s+(\d+)\s+"([^"]+)"\s*$', src, re.M)})
fid = {k for k, v in files.items() if v.endswith(a.file)}
m = re.search(r'^(\S*' + re.escape(a.kernel) + r'\S*):\s*;.*?\n(.*?)^\.Lfunc_end', src, re.S | re.M)
body = m.group(2).split('\n')
blocks = []
cur = {'name': 'entry', 'note': '', 'ins': [], 'lines': set()}
for ln in body:
    mm = re.match(r'^(\.LBB\S+|; %bb\.\d+):?\s*(;.*)?$', ln)
    if mm:
        blocks.append(cur)
        cur = {'name': mm.group(1), 'note': (mm.group(2) or '').strip('; ').strip(), 'ins': [], 'lines': set()}
        continue
    lm = re.match(r'^\s*\.loc\s+(\d+)\s+(\d+)', ln)
    if lm:
        if lm.group(1) in fid:
            cur['lines'].add(int(lm.group(2)))
        continue
    s = ln.strip()
    if ln.startswith('\t') and s and not s.startswith(('.', ';')):
        cur['ins'].append(s.split()[0])
blocks.append(cur)
tot = {'v': 0, 's': 0, 'mov': 0}
for b in blocks:
    ins = b['ins']
    v = sum(1 for i in ins if i.startswith('v_'))
    s = sum(1 for i in ins if i.startswith('s_'))
    mov = sum(1 for i in ins if i.startswith('v_mov_b32'))
    ds = sum(1 for i in ins if i.startswith('ds_'))
    vm = sum(1 for i in ins if i.startswith(('global_', 'buffer_', 'flat_', 'scratch_')))
    tot['v'] += v
    tot['s'] += s
    tot['mov'] += mov
    if a.all or mov >= a.min_mov:
        ls = sorted(b['lines'])
        print(f"{b['name']:12s} n={len(ins):4d} valu={v:4d} salu={s:4d} mov={mov:4d} ds={ds:3d} vmem={vm:3d} "
              f"[{b['note'][:40]}] lines={ls[:12]}{'...' if len(ls) > 12 else ''}")
print('total', tot, 'blocks', len(blocks))
