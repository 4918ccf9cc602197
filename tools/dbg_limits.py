import os, sys
sys.path.insert(0, os.getcwd()); sys.path.insert(0, os.path.join(os.getcwd(), 'tests'))
from oracle import oracle
oracle.build()
import test_errors as te
from test_gpu_parity import _diff
from fluidframework_amd.engine import MergeEngine
batch, bad = te._device_limit_batch(oracle)
clean, _ = te._device_limit_batch(oracle, faulty=False)
o = oracle.Oracle(clean.n_docs).apply(clean)
for b in (32, 0, 5, 1):
    eng = MergeEngine(batch.n_docs, ops_per_launch=b)
    eng.apply(batch)
    got = eng.checksums(); want = o.checksums()
    for d in range(8):
        if got[d] != want[d]:
            print('b', b, 'doc', d, eng.error(d), _diff(eng.state(d), o.state(d)))
    eng2 = MergeEngine(clean.n_docs, ops_per_launch=b)
    eng2.apply(clean)
    g2 = eng2.checksums()
    print('b', b, 'clean mismatches', [d for d in range(clean.n_docs) if g2[d] != want[d]])
