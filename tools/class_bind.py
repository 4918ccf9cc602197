#!/usr/bin/env python3
"""Which of mt_bin_kernel's fit conditions sets a document's capacity class at b ops per launch
(segments + empty blocks, leaf blocks, interior blocks, heap entries: mt_service.hip), measured on
the oracle's tree and heap at every launch boundary of a config's logs.  CPU only.
    python tools/class_bind.py [--config C3] [--docs 96] [--b 32]"""
import argparse
import collections
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)
from fluidframework_amd.oplog import CONFIGS, OpBatch  # noqa: E402
from oracle import oracle  # noqa: E402

# {CAP, LB, IB, H} of the register classes (mt_engine.cpp kClassParams)
CLS = [(128, 128, 40, 192), (192, 128, 40, 192)] + [(c, c // 2, c // 8 + 8, c // 2 + 64) for c in range(256, 1025, 64)]

ap = argparse.ArgumentParser()
ap.add_argument('--config', default='C3')
ap.add_argument('--docs', type=int, default=96)
ap.add_argument('--b', type=int, default=32)
a = ap.parse_args()
cfg = dict(CONFIGS[a.config])
cfg.pop('n_docs')
full = oracle.generate(a.docs, seed=7, **cfg)
o = oracle.Oracle(a.docs)
rp = full.row_ptr.astype(np.int64)
n_ops = cfg['ops_per_doc']
bind = collections.Counter()
slots = collections.Counter()
for t0 in range(0, n_ops, a.b):
    # every document's ops [t0, t0 + b) as one batch
    idx = np.concatenate([np.arange(rp[d] + t0, min(rp[d] + t0 + a.b, rp[d + 1])) for d in range(a.docs)])
    cnt = [max(0, min(a.b, int(rp[d + 1] - rp[d]) - t0)) for d in range(a.docs)]
    for d in range(a.docs):
        st = o.state(d)
        tree = st['tree']
        leaves = tree[-1] if tree else []
        nseg, nb0 = len(st['segs']), len(leaves)
        n_empty = sum(1 for c in leaves if c == 0)
        ib_need = max([len(L) for L in tree[:-1]], default=0) if len(tree) > 1 else 0
        heap = o.heap_size(d)
        k = cnt[d]
        conds = {
            'segments': lambda c: nseg + 2 * k + n_empty + 1 <= c[0],
            'leaf_blocks': lambda c: nb0 + 2 * k + 1 <= c[1],
            'interior': lambda c: ib_need + k + 1 <= c[2],
            'heap': lambda c: heap + 4 * k + 16 <= c[3],
        }
        first = {n: next((i for i, c in enumerate(CLS) if f(c)), len(CLS)) for n, f in conds.items()}
        cls = max(first.values())
        seg_cls = first['segments']
        if cls > seg_cls:
            bind[max(first, key=lambda n: first[n])] += 1
        else:
            bind['segments'] += 1
        slots['chosen'] += CLS[min(cls, len(CLS) - 1)][0]
        slots['by_segments'] += CLS[min(seg_cls, len(CLS) - 1)][0]
    sub = full.ops[idx]
    rows = np.concatenate([[0], np.cumsum(cnt)]).astype(np.uint32)
    o.apply(OpBatch(sub, full.payload, rows), threads=8)
tot = sum(bind.values())
print({k: round(v / tot, 3) for k, v in bind.items()}, 'slot cost chosen / by segments only:',
      round(slots['chosen'] / slots['by_segments'], 3))
