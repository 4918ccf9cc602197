#!/usr/bin/env python3
"""Summarise a rocprofv3 SQLite result (rocpd schema, ROCm 7.x) without extra tools:

  kernel stats  -- the same columns as `rocprofv3 --stats` (Name, Calls, TotalDurationNs,
                   AverageNs, Percentage, MinNs, MaxNs) plus the dispatch's VGPR/AGPR/SGPR counts;
  PMC totals    -- every counter of a --pmc pass summed per kernel (and per dispatch on average).

usage: rocpd_summary.py RESULTS.db [--csv OUT.csv] [--pmc]
"""
import argparse
import csv
import sqlite3
import sys
from collections import defaultdict


def kernel_stats(c):
    q = """select s.kernel_name, d.end - d.start, s.arch_vgpr_count, s.accum_vgpr_count, s.sgpr_count
           from rocpd_kernel_dispatch d join rocpd_info_kernel_symbol s on d.kernel_id = s.id"""
    acc = defaultdict(list)
    regs = {}
    for name, dur, vg, ag, sg in c.execute(q):
        acc[name].append(dur)
        regs[name] = (vg, ag, sg)
    total = sum(sum(v) for v in acc.values()) or 1
    rows = []
    for name, v in sorted(acc.items(), key=lambda kv: -sum(kv[1])):
        rows.append({'Name': name, 'Calls': len(v), 'TotalDurationNs': sum(v), 'AverageNs': sum(v) / len(v),
                     'Percentage': 100.0 * sum(v) / total, 'MinNs': min(v), 'MaxNs': max(v),
                     'VGPR': regs[name][0], 'AGPR': regs[name][1], 'SGPR': regs[name][2]})
    return rows


def pmc_totals(c):
    names = {pid: n for pid, n in c.execute('select id, name from rocpd_info_pmc')}
    q = """select s.kernel_name, p.pmc_id, sum(p.value), count(distinct d.id)
           from rocpd_pmc_event p join rocpd_kernel_dispatch d on p.event_id = d.event_id
           join rocpd_info_kernel_symbol s on d.kernel_id = s.id group by s.kernel_name, p.pmc_id"""
    out = defaultdict(dict)
    for kname, pid, val, nd in c.execute(q):
        out[kname][names.get(pid, pid)] = (val, nd)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('db')
    ap.add_argument('--csv')
    ap.add_argument('--pmc', action='store_true')
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = kernel_stats(c)
    cols = ['Name', 'Calls', 'TotalDurationNs', 'AverageNs', 'Percentage', 'MinNs', 'MaxNs', 'VGPR', 'AGPR', 'SGPR']
    w = csv.DictWriter(open(a.csv, 'w') if a.csv else sys.stdout, fieldnames=cols)
    w.writeheader()
    for r in rows:
        w.writerow(r)
    if a.pmc:
        for k, d in pmc_totals(c).items():
            print(k)
            for n, (v, nd) in sorted(d.items()):
                print(f'    {n:28s} total {v:16.0f}  per dispatch {v / max(1, nd):14.1f}')


if __name__ == '__main__':
    main()
