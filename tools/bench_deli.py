#!/usr/bin/env python3
"""Deli ticketing throughput on one MI355X (SURVEY.md §8 row a1, C5's per-GPU share).

Raw op messages of `--docs` documents x `--ops` ops (every client joined at seq 0) are derived
on the device from a synthetic C3-shaped op log; each step restores the documents' checkpoints
and tickets every message (mt_deli_ticket_device), optionally stamping seq / msn into the op
records (--stamp, the fused hand-off to the apply engine).  Prints one JSON line: messages/s,
the kernel's average duration (HIP events on the deli stream) and its HBM roofline fraction
with the algorithmic bytes: 16 B in + 16 B out per message (+ 12 B stamped per op record), and
9 B per client slot in + out per document."""
import argparse
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)

ap = argparse.ArgumentParser()
ap.add_argument('--docs', type=int, default=125000)
ap.add_argument('--ops', type=int, default=256)
ap.add_argument('--steps', type=int, default=5)
ap.add_argument('--stamp', action='store_true')
a = ap.parse_args()

import numpy as np  # noqa: E402

from fluidframework_amd.deli import RAW_DTYPE, TICKET_DTYPE, DeliSequencer, batch_device_ptrs  # noqa: E402
from fluidframework_amd.engine import MergeEngine  # noqa: E402
from fluidframework_amd.hipmem import DeviceBuffer  # noqa: E402
from fluidframework_amd.oplog import CONFIGS  # noqa: E402

cfg = dict(CONFIGS['C3'])
cfg.pop('n_docs')
cfg['ops_per_doc'] = a.ops
eng = MergeEngine(a.docs, ops_per_launch=32)
dev = eng.synthesize(seed=11, **cfg)
d_ops, _, d_row = batch_device_ptrs(dev)
n = dev.n_ops
msgs = DeviceBuffer(n * RAW_DTYPE.itemsize)
tick = DeviceBuffer(n * TICKET_DTYPE.itemsize)
dl = DeliSequencer(a.docs)
clients = {c: (0, 0, False) for c in range(1, cfg['n_clients'] + 1)}
dl.restore_all(seq=0, clients=clients)
dl.raw_from_ops(d_ops, d_row, a.docs, msgs.ptr)
dl.sync()
ms = []
t0 = time.perf_counter()
for _ in range(a.steps):
    dl.restore_all(seq=0, clients=clients)
    dl.ticket_device(msgs.ptr, d_row, a.docs, tick.ptr, d_ops if a.stamp else None, n)
    dl.sync()
    ms.append(dl.last_ms())
wall = time.perf_counter() - t0
t = tick.download(TICKET_DTYPE)
ok = bool(np.all(t['status'] == 1))
avg = sum(ms) / len(ms)
alg = n * (32 + (12 if a.stamp else 0)) + a.docs * 64 * 9 * 2 + a.docs * 20 * 2
print(json.dumps({
    'metric': 'deli tickets/sec (raw messages sequenced, 1 MI355X)', 'value': round(n / (avg * 1e-3), 1),
    'unit': 'msgs/s', 'docs': a.docs, 'msgs': n, 'kernel_ms': round(avg, 4), 'steps': a.steps,
    'wall_s': round(wall, 3), 'stamp': a.stamp, 'all_sent': ok,
    'roofline': {'bound': 'hbm', 'alg_bytes_per_launch': alg, 'achieved': round(alg / (avg * 1e-3) / 1e9, 1),
                 'peak': 8000.0, 'unit': 'GB/s', 'frac': round(alg / (avg * 1e-3) / 1e9 / 8000.0, 4)},
}), flush=True)
