#!/usr/bin/env python3
"""A/B helper for the delta-event path (bench.py's C3_events side line without the rest of the
bench): C3 on --docs documents with every callback recorded (mt_events_enable), one warm replay,
--reps timed replays (reset + apply of the HBM-resident logs; the drain is not timed), then the
per-class kernel times of a serialized replay.  One JSON line; MTGPU_LIB picks the build.
    python tools/bench_events.py [--docs 100000] [--reps 2]"""
import argparse
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)
from fluidframework_amd.engine import MergeEngine  # noqa: E402
from fluidframework_amd.hipmem import device_synchronize  # noqa: E402
from fluidframework_amd.oplog import CONFIGS  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument('--docs', type=int, default=100_000)
ap.add_argument('--reps', type=int, default=2)
a = ap.parse_args()
cfg = dict(CONFIGS['C3'])
cfg.pop('n_docs')
eng = MergeEngine(a.docs, ops_per_launch=32)
eng.enable_events(per_doc=8192)
dev = eng.synthesize(seed=1, **cfg)
gen = eng.checksums()
eng.drain_event_rows()
best = None
n_ev = 0
for r in range(a.reps + 1):
    eng.reset()
    device_synchronize()
    t0 = time.perf_counter()
    eng.apply_staged(dev)
    device_synchronize()
    el = time.perf_counter() - t0
    rows, rp = eng.drain_event_rows()
    n_ev = int(rp[-1])
    if r:
        best = el if best is None else min(best, el)
ok = bool(np.array_equal(eng.checksums(), gen))
eng.set_concurrent_classes(False)
eng.reset()
eng.apply_staged(dev)
eng.set_concurrent_classes(True)
cls = {hex(c): round(ms, 2) for c, ms, n, b in eng.last_class_stats() if n}
kern = {hex(c): eng.class_kernel(c) for c, ms, n, b in eng.last_class_stats() if n}
eng.drain_event_rows()
ops = a.docs * cfg['ops_per_doc']
print(json.dumps({'lib': os.environ.get('MTGPU_LIB', 'in-tree'), 'ops_per_s': round(ops / best, 1),
                  'ms_per_replay': round(best * 1e3, 2), 'events_per_replay': n_ev, 'replay_equals_generation': ok,
                  'class_ms_serialized': cls, 'kernels': kern}))
dev.free()
eng.close()
