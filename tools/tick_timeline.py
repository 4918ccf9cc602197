#!/usr/bin/env python3
"""Timeline of a host-fed submit (mt_submit_ticks) from a rocprofv3 trace with --kernel-trace and
--memory-copy-trace (rocpd SQLite): from the first large host -> device copy on, every copy and every
kernel, relative to that copy's start, with per-tick spans (bin kernel to the tick's last class
kernel) and the copies' achieved GB/s (diagnostic tooling).
    python tools/tick_timeline.py RESULTS.db [--min-mb 8] [--events 400] [--from-kernel restore_all --nth 2]"""
import argparse
import sqlite3


def cols(c, table):
    return [r[1] for r in c.execute(f'pragma table_info({table})')]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('db')
    ap.add_argument('--min-mb', type=float, default=8.0)
    ap.add_argument('--events', type=int, default=400)
    ap.add_argument('--from-kernel', default='', help='start at the --nth dispatch of a kernel whose name holds this')
    ap.add_argument('--nth', type=int, default=1)
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    tables = [r[0] for r in c.execute("select name from sqlite_master where type in ('table', 'view')")]
    mc = next((t for t in tables if t.startswith('rocpd_memory_copy')), None)
    ev = []
    for s, e, name in c.execute("""select d.start, d.end, s.kernel_name from rocpd_kernel_dispatch d
                                   join rocpd_info_kernel_symbol s on d.kernel_id = s.id"""):
        ev.append((s, e, 'K', name.split('(')[0][:60], 0))
    if mc:
        cc = cols(c, mc)
        size = 'size' if 'size' in cc else next((x for x in cc if 'size' in x or 'bytes' in x), None)
        name = 'name' if 'name' in cc else None
        q = f"select start, end, {size or 0}, {name or repr('copy')} from {mc}"
        for s, e, sz, nm in c.execute(q):
            ev.append((s, e, 'C', str(nm), int(sz or 0)))
    else:
        print('no memory-copy table in', tables)
    ev.sort()
    big = [x for x in ev if x[2] == 'C' and x[4] >= a.min_mb * 2**20]
    if not big:
        print('no copy of at least', a.min_mb, 'MiB')
        return
    t0 = big[0][0]
    if a.from_kernel:
        ks = [x for x in ev if x[2] == 'K' and a.from_kernel in x[3]]
        if len(ks) < a.nth:
            print('fewer than', a.nth, 'dispatches of', a.from_kernel)
            return
        t0 = ks[a.nth - 1][0]
    win = [x for x in ev if x[0] >= t0][:a.events]
    for s, e, kind, nm, sz in win:
        extra = f'{sz / 2**20:8.1f} MiB {sz / max(1, e - s):6.1f} GB/s' if kind == 'C' else ''
        print(f'{(s - t0) / 1e6:9.3f} {(e - t0) / 1e6:9.3f} ms  {kind} {nm:60s} {extra}')
    # GPU busy: the union of the window's kernel intervals
    ks = sorted((x[0], x[1]) for x in win if x[2] == 'K')
    busy_k, cur = 0, None
    for s, e in ks:
        if cur is None or s > cur[1]:
            if cur:
                busy_k += cur[1] - cur[0]
            cur = [s, e]
        else:
            cur[1] = max(cur[1], e)
    if cur:
        busy_k += cur[1] - cur[0]
    if ks:
        print(f'kernels: span {(ks[-1][1] - ks[0][0]) / 1e6:.2f} ms, busy {busy_k / 1e6:.2f} ms')
    copies = [x for x in win if x[2] == 'C' and x[4] >= a.min_mb * 2**20]
    if not copies:
        return
    tot = sum(x[4] for x in copies)
    span = max(x[1] for x in copies) - copies[0][0]
    busy = sum(x[1] - x[0] for x in copies)
    print(f'large copies: {len(copies)}, {tot / 2**30:.2f} GiB, span {span / 1e6:.1f} ms, busy {busy / 1e6:.1f} ms, '
          f'{tot / max(1, busy):.1f} GB/s while copying')


if __name__ == '__main__':
    main()
