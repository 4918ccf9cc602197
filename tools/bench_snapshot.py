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
print(json.dumps({'metric': 'snapshot extraction (SnapshotV1.extractSync), documents/sec, 1 MI355X',
                  'docs': a.docs, 'segments': segs, 'specs': nspec, 'kernel_ms': round(ms, 3),
                  'value': round(a.docs / (ms * 1e-3), 1), 'unit': 'docs/s',
                  'segments_per_s': round(segs / (ms * 1e-3), 1),
                  'host_emit': {'docs': a.sample, 'seconds': round(dt, 3), 'docs_per_s': round(a.sample / dt, 1),
                                'note': 'per-document readout + JSON on 1 host thread'}}), flush=True)
