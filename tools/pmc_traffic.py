#!/usr/bin/env python3
"""HBM traffic per launch of every kernel, from the two rocprofv3 PMC passes of
tools/rocprof.sh (FETCH_SIZE and WRITE_SIZE, in KiB per dispatch), corrected as
MI355X_MICROARCH.md's HBM section prescribes for gfx950: FETCH_SIZE reports half the bytes of
wide coalesced reads, so it is doubled; WRITE_SIZE is taken as is.

usage: pmc_traffic.py FETCH.db WRITE.db OUT.json
"""
import json
import re
import sqlite3
import subprocess
import sys
from collections import defaultdict


def per_dispatch(db, counter):
    c = sqlite3.connect(db)
    names = {pid for pid, n in c.execute('select id, name from rocpd_info_pmc') if n == counter}
    q = """select s.kernel_name, d.id, sum(p.value) from rocpd_pmc_event p
           join rocpd_kernel_dispatch d on p.event_id = d.event_id
           join rocpd_info_kernel_symbol s on d.kernel_id = s.id
           where p.pmc_id in (%s) group by d.id""" % ','.join(str(n) for n in names)
    acc = defaultdict(list)
    for kname, _, v in c.execute(q):
        acc[kname.removesuffix('.kd')].append(v * 1024.0)
    return acc


def short_name(mangled):
    """'void mtr::reg_apply_kernel<12>(...)' -> 'mtr::reg_apply_kernel<12>' (the names
    mt_class_kernel_name returns); the mangled name when no demangler is present."""
    try:
        d = subprocess.run(['c++filt', mangled], capture_output=True, text=True).stdout.strip()
    except OSError:
        return mangled
    d = re.sub(r'^void ', '', d)
    return d.split('(')[0] if '(' in d else d


def main():
    fetch = per_dispatch(sys.argv[1], 'FETCH_SIZE')
    write = per_dispatch(sys.argv[2], 'WRITE_SIZE')
    out = {}
    for k in sorted(set(fetch) | set(write)):
        f = sum(fetch.get(k, [])) / max(1, len(fetch.get(k, [])))
        w = sum(write.get(k, [])) / max(1, len(write.get(k, [])))
        out[short_name(k)] = {'mangled': k, 'fetch_bytes_per_launch_raw': f, 'write_bytes_per_launch': w,
                  'hbm_bytes_per_launch': 2.0 * f + w, 'launches': len(fetch.get(k, []))}
    meta = {'source': 'rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE passes of `bench.py --steps 1 --warmup 0 '
                      '--no-cpu-baseline` (tools/rocprof.sh)',
            'correction': 'hbm_bytes = 2 x FETCH_SIZE + WRITE_SIZE (gfx950 FETCH_SIZE counts half of wide reads)',
            'kernels': out}
    json.dump(meta, open(sys.argv[3], 'w'), indent=1)


if __name__ == '__main__':
    main()
