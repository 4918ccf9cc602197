#!/usr/bin/env python3
"""Static instruction mix of each kernel in a hipcc -S listing (diagnostic tooling)."""
import collections
import re
import sys

src = open(sys.argv[1]).read()
pat = sys.argv[2] if len(sys.argv) > 2 else ''
for m in re.finditer(r'^(\S+):\s*; @(\S+)\n(.*?)^\.Lfunc_end', src, re.S | re.M):
    name, body = m.group(1), m.group(3)
    if pat not in name:
        continue
    ins = [ln.split()[0] for ln in body.split('\n') if ln.startswith('\t') and ln.strip() and not ln.strip().startswith(('.', ';'))]
    c = collections.Counter(ins)
    valu = sum(v for k, v in c.items() if k.startswith('v_'))
    salu = sum(v for k, v in c.items() if k.startswith('s_'))
    print(name[:60], 'total', len(ins), 'valu', valu, 'salu', salu,
          'scratch', sum(v for k, v in c.items() if 'scratch' in k),
          'readlane', c['v_readlane_b32'], 'readfirstlane', c['v_readfirstlane_b32'], 'writelane', c['v_writelane_b32'],
          'cndmask', c['v_cndmask_b32_e64'] + c['v_cndmask_b32_e32'], 's_nop', c['s_nop'],
          'ds', sum(v for k, v in c.items() if k.startswith('ds_')), 'dpp', body.count('row_') + body.count('wave_'),
          'gpr_idx', c['s_set_gpr_idx_on'], 'waitcnt', c['s_waitcnt'], 'branches', sum(v for k, v in c.items() if k.startswith('s_cbranch')))
