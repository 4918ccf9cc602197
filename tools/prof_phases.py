#!/usr/bin/env python3
"""Diagnostic: per-phase cycle breakdown of the register apply engine (libmtgpu_prof.so, built
with `python fluidframework_amd/build.py --prof`).  Replays a synthetic config and prints, per
capacity class, the s_memtime cycles per op spent in each phase of RWave::apply."""
import argparse
import ctypes
import os
import sys

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault('MTGPU_LIB', os.path.join(HERE, 'fluidframework_amd', 'libmtgpu_prof.so'))
sys.path.insert(0, HERE)

from fluidframework_amd.engine import MergeEngine, lib  # noqa: E402
from fluidframework_amd.oplog import CONFIGS  # noqa: E402

SLOTS = ['load', 'scan', 'boundary', 'insert', 'range', 'zamboni', 'scour', 'store', 'ops', 'zpop', 'repack',
         'b_get', 'b_blk', 'b_txt', 'b_ins', 'n_scour', 'n_unlink', 'n_append', 'n_split', 'compact',
         'n_compact', 'n_appbytes', 'b_srch', 'b_leaf', 'op']
STRIDE = 32  # kProfStride in mt_apply_reg.hip

ap = argparse.ArgumentParser()
ap.add_argument('--config', default='C3')
ap.add_argument('--docs', type=int, default=20000)
ap.add_argument('--ops', type=int, default=0)
a = ap.parse_args()
cfg = dict(CONFIGS[a.config])
cfg.pop('n_docs')
if a.ops:
    cfg['ops_per_doc'] = a.ops
eng = MergeEngine(a.docs, ops_per_launch=32)
dev = eng.synthesize(seed=5, **cfg)
L = lib()
L.mt_prof_read.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
buf = (ctypes.c_ulonglong * (16 * STRIDE))()
L.mt_prof_read(buf, 16 * STRIDE)  # clear
eng.reset()
eng.apply_staged(dev)
L.mt_prof_read(buf, 16 * STRIDE)
for k in range(1, 17):
    v = list(buf[STRIDE * (k - 1):STRIDE * (k - 1) + len(SLOTS)])
    ops = v[SLOTS.index('ops')]
    if not ops:
        continue
    parts = ' '.join((f'{n}={v[i] / ops:.2f}' if n.startswith('n_') else f'{n}={v[i] / ops:.0f}') for i, n in enumerate(SLOTS)
                     if n != 'ops' and (v[i] or n.startswith('n_')))
    print(f'K={k:2d} ops={ops:10d} cycles/op: {parts}')
