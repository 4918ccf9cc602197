import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)


def pytest_configure(config):
    config.addinivalue_line('markers', 'gpu: needs an MI355X (runs on the GPU box via gpurun)')
    config.addinivalue_line('markers', 'reference: needs /root/reference + node (build container only)')


GOLDEN = os.path.join(REPO, 'tests', 'golden')
GOLDEN_SETS = ['scenarios', 'markers', 'synth_c1', 'synth_c2', 'synth_c3', 'synth_c4', 'synth_tiny', 'synth_markers']
# beyond the narrow limits (include/mtgpu.h "limits"): UTF-16 text, > 100 client ids, u16 value ids,
# keys 8..15 -- tests/golden/make_wide.py
WIDE_SETS = ['wide', 'wide_synth', 'wide_many', 'wide_xl']


# reference pins at the benchmark configs' full shape (tests/golden/make_fullshape.py): the logs are
# regenerated from the recorded config and seed, their bytes checked against the recorded SHA-256
FULLSHAPE_SETS = ['full_c3', 'full_c4', 'full_c5', 'full_c3w', 'fuzz_1k']


def load_fullshape(name):
    """(batch, fixture) of a full-shape set: the regenerated log, proven to be the bytes the
    reference replayed, and the reference's per-document results."""
    import json
    from oracle import oracle
    sys.path.insert(0, GOLDEN)
    from make_fullshape import log_sha256
    with open(os.path.join(GOLDEN, name + '.json')) as f:
        fx = json.load(f)
    oracle.build()
    batch = oracle.generate(fx['n_docs'], seed=fx['seed'], **fx['cfg'])
    assert log_sha256(batch) == fx['log_sha256'], f'{name}: the generator no longer produces the pinned log'
    return batch, fx


def load_golden(name):
    import json
    from fluidframework_amd.oplog import OpBatch
    batch = OpBatch.load(os.path.join(GOLDEN, name + '.mtlog'))
    with open(os.path.join(GOLDEN, name + '.expected.jsonl')) as f:
        exp = [json.loads(line) for line in f if line.strip()]
    return batch, exp


@pytest.fixture(scope='session')
def oracle_lib():
    from oracle import oracle
    oracle.build()
    return oracle
