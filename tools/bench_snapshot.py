#!/usr/bin/env python3
"""Snapshot extraction throughput: C3-shaped documents after a full
replay; the device pass of SnapshotV1.extractSync over every document in one launch
(mt_snapshot_extract), and the host JSON emit of a sample (mt_get_snapshot)."""
import argparse
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)
ap = argparse.ArgumentParser()
ap.add_argument('--docs', type=int, default=100000)
ap.add_argument('--sample', type=int, default=2000)
ap.add_argument('--batch', type=int, default=4096)
a = ap.parse_args()
from fluidframework_amd.engine import MergeEngine  # noqa: E402
from fluidframework_amd.oplog import CONFIGS  # noqa: E402

cfg = dict(CONFIGS['C3'])
cfg.pop('n_docs')
eng = MergeEngine(a.docs, ops_per_launch=32)
eng.synthesize(seed=17, **cfg)            # documents end in the post-generation state
eng.snapshot_extract()                    # warm-up
ms, nspec = eng.snapshot_extract()
segs = int(eng.seg_counts().sum())
names = ['observer'] + ['c%d' % i for i in range(1, 64)]
t0 = time.perf_counter()
nbytes = 0
for d in range(a.sample):
    nbytes += len(json.dumps(eng.snapshot(d, 0, names)))
dt = time.perf_counter() - t0
# the batched form: every document's JSON on all host cores (mt_get_snapshots), in slices
t1 = time.perf_counter()
bbytes = 0
for d0 in range(0, a.docs, a.batch):
    raw, off = eng.snapshots_raw(d0, min(a.batch, a.docs - d0), 0, names)
    bbytes += len(raw)
bdt = time.perf_counter() - t1
print(json.dumps({'metric': 'snapshot extraction (SnapshotV1.extractSync), documents/sec, 1 MI355X',
                  'docs': a.docs, 'segments': segs, 'specs': nspec, 'kernel_ms': round(ms, 3),
                  'value': round(a.docs / (ms * 1e-3), 1), 'unit': 'docs/s',
                  'segments_per_s': round(segs / (ms * 1e-3), 1),
                  'host_emit': {'docs': a.sample, 'seconds': round(dt, 3), 'docs_per_s': round(a.sample / dt, 1),
                                'note': 'per-document readout + JSON on 1 host thread'},
                  'host_emit_batched': {'docs': a.docs, 'seconds': round(bdt, 3), 'docs_per_s': round(a.docs / bdt, 1),
                                        'bytes': bbytes, 'batch': a.batch,
                                        'note': 'mt_get_snapshots: one extraction launch + one copy per array per '
                                                'batch, JSON on up to 16 host threads'}}), flush=True)
