#!/usr/bin/env python3
"""The editing-client farm side line (bench.py slow_paths.editing_farm) at several records-per-launch
settings: how much of the editing form's time is per-launch document staging (load / store of the
document's structure) and how much is per-record apply.  Prints one line per setting."""
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)


def main():
    from fluidframework_amd.engine import MergeEngine
    from fluidframework_amd.hipmem import device_synchronize
    from fluidframework_amd.oplog import OpBatch
    n_docs = int(sys.argv[1]) if len(sys.argv) > 1 else 100000
    src = OpBatch.load(os.path.join(HERE, 'tests', 'golden', 'local_big.mtlog'))
    lens = np.diff(src.row_ptr.astype(np.int64))
    pick = np.arange(n_docs) % src.n_docs
    starts = src.row_ptr[:-1].astype(np.int64)[pick]
    rp = np.concatenate([[0], np.cumsum(lens[pick])]).astype(np.int64)
    idx = np.repeat(starts - rp[:-1], lens[pick]) + np.arange(rp[-1])
    batch = OpBatch(src.ops[idx], src.payload, rp.astype(np.uint32))
    n_rec = int(rp[-1])
    ref = None
    for b in [int(x) for x in (sys.argv[2] if len(sys.argv) > 2 else '32,128,0').split(',')]:
        eng = MergeEngine(n_docs, ops_per_launch=b)
        dev = eng.stage(batch)
        eng.reset()
        eng.apply_staged(dev)
        device_synchronize()
        t0 = time.perf_counter()
        eng.reset()
        eng.apply_staged(dev)
        device_synchronize()
        el = time.perf_counter() - t0
        eng.set_concurrent_classes(False)
        eng.reset()
        eng.apply_staged(dev)
        cls = eng.last_class_stats()
        cs = eng.checksums()
        same = ref is None or bool(np.array_equal(cs, ref))
        ref = cs if ref is None else ref
        # (a sum: the farm tiles 16 source documents, so an xor of the checksums would cancel)
        digest = int(np.add.reduce(cs.astype(np.uint64), dtype=np.uint64))
        used = [(hex(c), round(ms, 2), n) for c, ms, n, _ in cls if n]
        print(f'b={b}: {n_rec / el / 1e6:.1f} M records/s ({el * 1e3:.1f} ms), classes {used}, '
              f'checksums agree {same}, digest {digest:016x}', flush=True)
        dev.free()
        eng.close()


if __name__ == '__main__':
    main()
