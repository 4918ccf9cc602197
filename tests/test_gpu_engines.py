"""Both device engines against the CPU oracle on workloads that push them into their corners:
documents that shrink to nothing (empty leaf blocks, packs, the register engine's padding slots),
documents with more than 32 clients (routed to the LDS engine), every capacity class, several
launch sizes; and the two engines against each other.  Run on the GPU box:
python -m pytest tests -m gpu"""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

WORKLOADS = {
    # removes outpace inserts: documents repeatedly shrink towards empty
    'shrink': dict(n_clients=8, ops_per_doc=1536, max_lag=16, p_insert=0.3, p_remove=0.7),
    # 48 clients: overlap sets need 64 bits, so these documents run on the LDS engine
    'wide': dict(n_clients=48, ops_per_doc=768, max_lag=24, n_keys=4, n_values=8, p_insert=0.5, p_remove=0.3,
                 p_overlap=0.4, p_insert_props=0.2),
    # annotate-heavy with a wide window: property runs block zamboni appends
    'annotate': dict(n_clients=16, ops_per_doc=1024, max_lag=64, n_keys=8, n_values=4, p_insert=0.4,
                     p_remove=0.15, p_overlap=0.3, p_null=0.2, p_rewrite=0.1, p_insert_props=0.3),
    # insert-heavy: documents grow through every capacity class
    'grow': dict(n_clients=4, ops_per_doc=2048, max_lag=4, n_keys=2, n_values=3, p_insert=0.85, p_remove=0.1,
                 p_insert_props=0.5),
}


def _engine(n, b, engine=None):
    from fluidframework_amd.engine import MergeEngine
    old = os.environ.get('MTGPU_ENGINE')
    try:
        if engine:
            os.environ['MTGPU_ENGINE'] = engine
        else:
            os.environ.pop('MTGPU_ENGINE', None)
        return MergeEngine(n, ops_per_launch=b)
    finally:
        if old is None:
            os.environ.pop('MTGPU_ENGINE', None)
        else:
            os.environ['MTGPU_ENGINE'] = old


@pytest.mark.parametrize('b', [32, 7])
@pytest.mark.parametrize('name', sorted(WORKLOADS))
def test_workload_against_oracle(oracle_lib, name, b):
    n = 128
    batch = oracle_lib.generate(n, seed=4242, **WORKLOADS[name])
    want = oracle_lib.Oracle(n).apply(batch, threads=8).checksums()
    eng = _engine(n, b)
    eng.apply(batch)
    got = eng.checksums()
    bad = np.nonzero(want != got)[0]
    assert not len(bad), f'{len(bad)}/{n} docs differ, first {int(bad[0])}: err={eng.error(int(bad[0]))}'
    assert all(eng.error(d) == (0, 0) for d in range(n))


def test_engines_agree():
    """The register engine and the LDS engine end in the same state on the same log."""
    from fluidframework_amd.oplog import CONFIGS
    from oracle import oracle
    cfg = dict(CONFIGS['C3'])
    cfg.pop('n_docs')
    cfg['ops_per_doc'] = 512
    n = 192
    batch = oracle.generate(n, seed=77, **cfg)
    sums = []
    for engine in (None, 'lds'):
        eng = _engine(n, 32, engine)
        eng.apply(batch)
        sums.append(eng.checksums())
    assert np.array_equal(sums[0], sums[1])


def test_concurrent_classes_match_serialized(oracle_lib):
    """The capacity classes of a tick run on their own streams by default; serializing them
    (mt_set_concurrent_classes(eng, 0)) must give the same state, and both the oracle's.  A mix
    of growing documents and > 32-client documents puts several classes (and both engines) into
    the same ticks."""
    n = 96
    grow = oracle_lib.generate(n, seed=31, **WORKLOADS['grow'])
    want = oracle_lib.Oracle(n).apply(grow, threads=8).checksums()
    sums = []
    for concurrent in (True, False):
        eng = _engine(n, 16)
        eng.set_concurrent_classes(concurrent)
        eng.apply(grow)
        sums.append(eng.checksums())
        classes = [cap for cap, _, launches, _ in eng.last_class_stats() if launches]
        assert len(classes) >= 3, classes
    assert np.array_equal(sums[0], sums[1])
    assert np.array_equal(sums[0], want)


def test_wide_client_documents_use_the_c64_register_form(oracle_lib):
    """Documents with client ids above 32 run on the register engine's C64 form (a second overlap
    register per slot: MT_CLASS_C64 | capacity in the class stats, mtr::reg_apply_kernel_c64<K>), at
    the capacity of the class they fit, not on the LDS engine at 2048 segments; label-key documents
    keep the LDS engine at their class's capacity (MT_CLASS_LDS)."""
    n = 64
    batch = oracle_lib.generate(n, seed=5150, **WORKLOADS['wide'])
    want = oracle_lib.Oracle(n).apply(batch, threads=8).checksums()
    eng = _engine(n, 32)
    eng.apply(batch)
    assert np.array_equal(eng.checksums(), want)
    used = {cap: launches for cap, _, launches, _ in eng.last_class_stats() if launches}
    c64 = sorted(cap & ~0x10000000 for cap in used if cap & 0x10000000)
    assert c64 and c64[0] < 1024, used
    assert 2048 not in used, used
    assert eng.class_kernel(0x10000000 | c64[0]) == 'mtr::reg_apply_kernel_c64<%d>' % (c64[0] // 64)
    # the same documents with declared label keys: the LDS engine at the register classes' capacities
    eng2 = _engine(n, 32)
    eng2.set_label_keys(6, 7)
    eng2.apply(batch)
    assert np.array_equal(eng2.checksums(), want)
    used2 = {cap: launches for cap, _, launches, _ in eng2.last_class_stats() if launches}
    assert any(cap & 0x20000000 for cap in used2) and not any(cap & 0x10000000 for cap in used2), used2
