#!/usr/bin/env python3
"""Editing-client throughput: the reference farm's local_big logs (one
editing client's view: local edits, remote ops, acks; tests/golden/make_local.py) tiled over many
documents and applied in one batch on the device's editing form, with the CPU oracle's time on a
sample of the same documents beside it.  Records per second counts every record (local edits,
remote ops and acks)."""
import argparse
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)
ap = argparse.ArgumentParser()
ap.add_argument('--docs', type=int, default=32768)
ap.add_argument('--reps', type=int, default=3)
ap.add_argument('--cpu-docs', type=int, default=256)
a = ap.parse_args()
from fluidframework_amd.engine import MergeEngine  # noqa: E402
from fluidframework_amd.oplog import OpBatch  # noqa: E402

src = OpBatch.load(os.path.join(HERE, 'tests', 'golden', 'local_big.mtlog'))
lens = np.diff(src.row_ptr.astype(np.int64))
pick = np.arange(a.docs) % src.n_docs
idx = np.concatenate([np.arange(int(src.row_ptr[p]), int(src.row_ptr[p + 1])) for p in pick])
rp = np.concatenate([[0], np.cumsum(lens[pick])]).astype(np.uint32)
batch = OpBatch(src.ops[idx].copy(), src.payload, rp)
n = int(rp[-1])
best = None
for r in range(a.reps):
    eng = MergeEngine(a.docs, ops_per_launch=32)
    t0 = time.perf_counter()
    eng.apply(batch)
    dt = time.perf_counter() - t0
    errs = sum(1 for d in range(0, a.docs, 97) if eng.error(d) != (0, 0))
    eng.close()
    best = dt if best is None else min(best, dt)
cpu = None
try:
    from oracle import oracle
    sub = OpBatch(src.ops[np.concatenate([np.arange(int(src.row_ptr[p]), int(src.row_ptr[p + 1]))
                                          for p in pick[:a.cpu_docs]])].copy(), src.payload,
                  np.concatenate([[0], np.cumsum(lens[pick[:a.cpu_docs]])]).astype(np.uint32))
    t0 = time.perf_counter()
    oracle.Oracle(sub.n_docs).apply(sub, threads=1)
    cpu = int(sub.row_ptr[-1]) / (time.perf_counter() - t0)
except Exception as e:  # the oracle is optional here
    print('oracle unavailable:', e, file=sys.stderr)
print(json.dumps({'metric': 'editing-client records applied/sec (local edits + remote ops + acks)',
                  'docs': a.docs, 'records': n, 'best_s': round(best, 4), 'value': round(n / best, 1),
                  'errors_sampled': errs, 'cpu_oracle_1thread_records_per_s': None if cpu is None else round(cpu, 1),
                  'source': 'tests/golden/local_big.mtlog tiled (reference farm logs), apply incl. H2D of the records'}))
