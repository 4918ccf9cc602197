#!/usr/bin/env python3
"""Per class: algorithmic bytes per launch (the bench line's roofline.classes) against the PMC HBM bytes
per launch (tools/pmc_traffic.py output of the same command), and their ratio.
    python tools/pmc_classes.py BENCH_LINE.json PMC.json"""
import json
import sys


def main(bench, pmc):
    line = json.loads([x for x in open(bench).read().split('\n') if x.startswith('{')][-1])
    ks = json.load(open(pmc))['kernels']
    cl = line['roofline']['classes']
    tot = sum(v['ms'] for v in cl.values()) or 1
    print(f"{'class':>10} {'kernel':34} {'ms':>8} {'share':>6} {'alg MB':>8} {'pmc MB':>8} {'ratio':>6}")
    for label, v in cl.items():
        k = v['kernel']
        p = ks.get(k)
        if p is None:
            hit = [x for n, x in ks.items() if n.startswith(k[:-1] + ', ')]
            p = hit[0] if len(hit) == 1 else None
        pb = p['hbm_bytes_per_launch'] if p else None
        alg = v['alg_bytes_per_launch']
        print(f"{label:>10} {k:34} {v['ms']:8.2f} {v['ms'] / tot:6.3f} {alg / 1e6:8.1f} "
              f"{(pb or 0) / 1e6:8.1f} {(pb / alg if pb and alg else 0):6.2f}")


if __name__ == '__main__':
    main(sys.argv[1], sys.argv[2])
