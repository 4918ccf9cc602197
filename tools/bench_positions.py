#!/usr/bin/env python3
"""Microbench of the device position queries (mt_resolve_positions_device; include/mtgpu.h): 1M
getContainingSegment queries in the local view, plus getPosition-by-ordinal queries, over C3
documents replayed on the device, queries and results resident in HBM.  Prints one JSON line
(queries/s, the kernel's time, the bytes it reads).  Run on the GPU box:
    python tools/bench_positions.py [--docs 20000] [--queries 1000000]"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)

from fluidframework_amd.engine import (POS_CONTAINING, POS_LOCAL, POS_OF_ORDINAL, POS_QUERY_DTYPE,  # noqa: E402
                                       POS_RESULT_DTYPE, MergeEngine, _check, lib)
from fluidframework_amd.hipmem import DeviceBuffer, hip  # noqa: E402
from fluidframework_amd.oplog import CONFIGS  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument('--docs', type=int, default=20000)
ap.add_argument('--queries', type=int, default=1_000_000)
ap.add_argument('--reps', type=int, default=5)
a = ap.parse_args()
cfg = dict(CONFIGS['C3'])
cfg.pop('n_docs')
eng = MergeEngine(a.docs, ops_per_launch=32)
dev = eng.synthesize(seed=11, **cfg)
lens = np.array([eng.length(d) for d in range(a.docs)], dtype=np.int64)
rng = np.random.default_rng(5)
q = np.zeros(a.queries, dtype=POS_QUERY_DTYPE)
q['doc'] = rng.integers(0, a.docs, a.queries)
q['pos'] = (rng.random(a.queries) * (lens[q['doc']] + 1)).astype(np.int32)
q['ref_seq'] = POS_LOCAL
q['kind'] = POS_CONTAINING
half = a.queries // 2  # the second half: getPosition of the segments the first half found
dq = DeviceBuffer(q.nbytes).upload(q)
dr = DeviceBuffer(a.queries * POS_RESULT_DTYPE.itemsize)
L = lib()


def run(qbuf, n):
    _check(L.mt_resolve_positions_device(eng.h, ctypes.c_void_p(qbuf.ptr), n, ctypes.c_void_p(dr.ptr)),
           'mt_resolve_positions_device')
    hip().hipDeviceSynchronize()


run(dq, a.queries)  # warm
times = []
for _ in range(a.reps):
    t0 = time.perf_counter()
    run(dq, a.queries)
    times.append(time.perf_counter() - t0)
res = dr.download(POS_RESULT_DTYPE, a.queries)
# the host entry point on a sample must agree
k = 4096
host = eng.resolve_positions(q[:k])
assert np.array_equal(host, res[:k]), 'device-resident and host-staged queries differ'
# getPosition-by-ordinal of the found segments: every position must come back
q2 = q[:half].copy()
found = res[:half]['ordinal'] >= 0
q2['pos'] = np.where(found, res[:half]['ordinal'], 0)
q2['kind'] = POS_OF_ORDINAL
dq2 = DeviceBuffer(q2.nbytes).upload(q2)
t0 = time.perf_counter()
run(dq2, half)
t_ord = time.perf_counter() - t0
res2 = dr.download(POS_RESULT_DTYPE, half)
assert np.array_equal(res2['position'][found], res[:half]['position'][found])
assert np.all(res[:a.queries]['ordinal'][q['pos'] < lens[q['doc']]] >= 0)
best = min(times)
print(json.dumps({'queries': a.queries, 'docs': a.docs, 'config': 'C3 (1024 ops)',
                  'containing_queries_per_s': round(a.queries / best, 1), 'ms_per_batch': round(best * 1e3, 3),
                  'ordinal_queries_per_s': round(half / t_ord, 1),
                  'mean_doc_length_chars': round(float(lens.mean()), 1),
                  'note': 'one wave per query; wall time of the launch incl. synchronize; queries and results in HBM'}))
for b in (dq, dr, dq2):
    b.free()
dev.free()
eng.close()
