"""An editing client whose document grows past the editing form's LDS capacity (MT_LOC_CAP = 1024
segments): the editing form's HBM-workspace classes (mt_apply.hip apply_kernel_g<CAP, false, true>,
mt_launch_apply_loc_big; include/mtgpu.h MT_SEQ_LOCAL).

Pinned by the reference itself: tests/golden/local_huge.expected.jsonl holds the canonical states
of a reference Client c1 replaying local_huge.mtlog (tests/golden/make_local_huge.py: the
local_farm.js farm of reference clients, 32000 edits over 4 clients, c1 lagging), at checkpoints
and at the end; both documents pass 1024 segments (up to 1609) with edits pending throughout."""
import json
import os

import pytest

from conftest import GOLDEN
from test_local import checkpoint_batch, prefix

NAME = 'local_huge'


def load_rows():
    with open(os.path.join(GOLDEN, NAME + '.expected.jsonl')) as f:
        return [json.loads(line) for line in f]


def test_fixture_grows_past_the_lds_capacity():
    from fluidframework_amd.oplog import OpBatch
    rows = load_rows()
    assert all(r['err'] is None for r in rows)
    assert all(max(len(st['segs']) for _, st in r['states']) > 1024 for r in rows)
    mid = [st for r in rows for _, st in r['states'][:-1]]
    assert sum(1 for st in mid for s in st['segs'] if s[1] == -1) > 0  # pending inserts at checkpoints
    b = OpBatch.load(os.path.join(GOLDEN, NAME + '.mtlog'))
    local = b.ops['seq'] == -1
    assert local.sum() > 5000 and (b.ops['client'][~local] == 1).sum() == local.sum()  # every edit acked


def test_oracle_editing_client_matches_reference_past_1024_segments(oracle_lib):
    from fluidframework_amd.oplog import OpBatch
    batch = OpBatch.load(os.path.join(GOLDEN, NAME + '.mtlog'))
    o = oracle_lib.Oracle(batch.n_docs).apply(batch)
    for r in load_rows():
        d = r['doc']
        assert o.error(d) == (0, 0), (d, o.error(d))
        assert o.state(d) == r['states'][-1][1], d
        for k, want in r['states'][-3:-1]:
            assert oracle_lib.Oracle(1).apply(prefix(batch, d, k)).state(0) == want, (d, k)


@pytest.mark.gpu
@pytest.mark.parametrize('b', [1, 32])
def test_engine_editing_form_past_1024_segments_matches_reference(b):
    """Every checkpoint state and the final state equal the reference's; the documents past 1024
    segments ran on the editing form's 2048-slot HBM-workspace class (class stats
    MT_CLASS_EDITING | 2048, mt::apply_kernel_g<2048, false, true>)."""
    from fluidframework_amd.engine import MergeEngine
    from fluidframework_amd.oplog import OpBatch
    batch = OpBatch.load(os.path.join(GOLDEN, NAME + '.mtlog'))
    rows = load_rows()
    editing_g = 0x40000000 | 2048
    for q in range(len(rows[0]['states'])):
        cb = checkpoint_batch(batch, rows, q)
        eng = MergeEngine(cb.n_docs, ops_per_launch=b)
        eng.apply(cb)
        used = {cap: n for cap, _, n, _ in eng.last_class_stats() if n}
        for i, r in enumerate(rows):
            assert eng.error(i) == (0, 0), (r['doc'], q, eng.error(i))
            assert eng.state(i) == r['states'][q][1], (r['doc'], q, b)
        if max(len(r['states'][q][1]['segs']) for r in rows) > 1024 + 2 * b:
            assert used.get(editing_g, 0) > 0, used
            assert eng.class_kernel(editing_g) == 'mt::apply_kernel_g<2048, false, true>'
        eng.close()
