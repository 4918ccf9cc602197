"""Snapshot emit on the CPU: the restatement oracle/snapshot.py of
SnapshotV1.extractSync + emit (snapshotV1.ts:57-247), applied to the oracle's replayed states,
against the trees the reference itself emitted for the same logs (tests/golden/*.snapshot*.jsonl,
written by tests/golden/make_snapshots.py)."""
import json
import os

import pytest

from conftest import GOLDEN

SETS = [('scenarios', None), ('synth_c1', None), ('synth_c3', None), ('synth_c4', None), ('synth_tiny', None),
        ('markers', None), ('synth_markers', None),
        ('synth_c3', 300)]


def load_snapshots(name, chunk=None):
    path = os.path.join(GOLDEN, name + ('.snapshot%d' % chunk if chunk else '.snapshot') + '.jsonl')
    with open(path) as f:
        return [json.loads(x) for x in f if x.strip()]


@pytest.mark.parametrize('name,chunk', SETS)
def test_restatement_matches_reference_snapshots(oracle_lib, name, chunk):
    from fluidframework_amd.oplog import OpBatch
    from oracle import snapshot
    batch = OpBatch.load(os.path.join(GOLDEN, name + '.mtlog'))
    o = oracle_lib.Oracle(batch.n_docs).apply(batch)
    want = load_snapshots(name, chunk)
    assert len(want) == batch.n_docs
    for d, w in enumerate(want):
        got = snapshot.emit(o.state(d), chunk or snapshot.DEFAULT_CHUNK)
        assert got == w['snapshot'], (name, d)
