#!/usr/bin/env python3
"""Host gaps between the ticks of an apply, from a rocprofv3 kernel trace (rocpd SQLite): for every
mt_bin_kernel dispatch, the idle time of the GPU just before it (the previous tick's last kernel
end -> this bin's start: the host waiting on the previous tick and launching this one) and just after
it (bin end -> the first class kernel's start: the count copy, the host's wake-up and its launches).
Copy kernels (rocclr) count as busy.  Prints the totals and per-tick medians (diagnostic tooling).
    python tools/tick_gaps.py RESULTS.db"""
import sqlite3
import statistics
import sys


def main(db):
    c = sqlite3.connect(db)
    rows = sorted(c.execute("""select d.start, d.end, s.kernel_name from rocpd_kernel_dispatch d
                               join rocpd_info_kernel_symbol s on d.kernel_id = s.id"""))
    bins = [i for i, r in enumerate(rows) if 'mt_bin_kernel' in r[2]]
    before, after = [], []
    for n, i in enumerate(bins):
        if n:
            prev_end = max(r[1] for r in rows[bins[n - 1]:i])
            before.append(max(0, rows[i][0] - prev_end))
        nxt = bins[n + 1] if n + 1 < len(bins) else len(rows)
        later = [r for r in rows[i + 1:nxt] if 'apply_kernel' in r[2]]
        if later:
            after.append(max(0, min(r[0] for r in later) - rows[i][1]))
    bin_ns = [rows[i][1] - rows[i][0] for i in bins]
    span = rows[-1][1] - rows[0][0]
    print(f'bins {len(bins)}  trace span {span / 1e6:.1f} ms')
    print(f'idle before bin: total {sum(before) / 1e6:.2f} ms, median {statistics.median(before or [0]) / 1e3:.1f} us')
    print(f'idle bin -> first class kernel: total {sum(after) / 1e6:.2f} ms, '
          f'median {statistics.median(after or [0]) / 1e3:.1f} us')
    print(f'bin kernel: total {sum(bin_ns) / 1e6:.2f} ms, median {statistics.median(bin_ns or [0]) / 1e3:.1f} us')


if __name__ == '__main__':
    main(sys.argv[1])
