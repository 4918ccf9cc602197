"""Range stacks: Client.getStackContext(startPos, rangeLabels)
(client.ts:946-948 -> mergeTree.ts:1750-1760) for the own client, pinned by the reference itself:
tests/golden/stacks.expected.jsonl holds the stacks the reference's observer Client returned on the
tiles_* logs (tests/golden/make_tiles.py) with range labels on property key 1 ("referenceRangeLabels",
value id v = the labels L<i> of its bits i, js/mtlog.js tileLabels) -- nested / unmatched / removed
NestBegin and NestEnd markers and marker-heavy synthetic logs.  The oracle restates search with
recordRangeLeaf / rangeShift over its pointer tree; the engine answers a batch of queries on the
device (mt_range_stacks)."""
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN
from test_tiles import LOGS, label_mask

RANGE_KEY = 1


def load_stacks():
    out = {}
    with open(os.path.join(GOLDEN, 'stacks.expected.jsonl')) as f:
        for line in f:
            r = json.loads(line)
            out.setdefault(r['log'], []).append(r)
    return out


def test_fixture_covers_nesting_and_unmatched_ends():
    ans = [a for v in load_stacks().values() for r in v for a in r['answers']]
    stacks = [a[2] for a in ans]
    assert sum(1 for s in stacks if s) > 300
    assert any(len(s) >= 3 for s in stacks)
    assert any(s and s[0][1] == 4 for s in stacks)  # an unmatched end at the bottom
    assert any(len(s) >= 2 and s[0][1] == 4 and s[-1][1] == 2 for s in stacks)  # ends then begins


@pytest.mark.parametrize('name', LOGS)
def test_oracle_stack_context_matches_reference(oracle_lib, name):
    from fluidframework_amd.oplog import OpBatch
    batch = OpBatch.load(os.path.join(GOLDEN, name + '.mtlog'))
    o = oracle_lib.Oracle(batch.n_docs).apply(batch)
    masks = [label_mask(k) for k in range(4)]
    for r in load_stacks()[name]:
        for pos, lab, want in r['answers']:
            assert o.stack_context(r['doc'], pos, RANGE_KEY, masks[lab]) == want, (name, r['doc'], pos, lab)


def _as_lists(stacks):
    return [[[int(x['pos']), int(x['ref_type'])] for x in s] for s in stacks]


@pytest.mark.gpu
@pytest.mark.parametrize('name', LOGS)
def test_engine_range_stacks_match_reference(name):
    from fluidframework_amd.engine import TILE_QUERY_DTYPE, MergeEngine
    from fluidframework_amd.oplog import OpBatch
    batch = OpBatch.load(os.path.join(GOLDEN, name + '.mtlog'))
    eng = MergeEngine(batch.n_docs, ops_per_launch=16)
    eng.set_label_keys(0, 1)  # (tile labels on key 0, range labels on key 1)
    eng.apply(batch)
    rows = load_stacks()[name]
    masks = [label_mask(k) for k in range(4)]
    q = np.array([(r['doc'], pos, RANGE_KEY, 0, 0, 0, masks[lab].view('<u4'), 0)
                  for r in rows for pos, lab, _ in r['answers']], dtype=TILE_QUERY_DTYPE)
    want = [a[2] for r in rows for a in r['answers']]
    got = _as_lists(eng.range_stacks(q, cap=2))  # deeper stacks take the re-ask path
    bad = [i for i in range(len(want)) if got[i] != want[i]]
    assert not bad, [(q[i]['doc'], q[i]['pos'], got[i], want[i]) for i in bad[:5]]


@pytest.mark.gpu
def test_engine_range_stacks_match_oracle_on_fuzz(oracle_lib):
    """Marker-heavy fuzz (with zamboni): every position of every document, every label; the
    stack's ordinals name markers of the document."""
    from fluidframework_amd.engine import TILE_QUERY_DTYPE, MergeEngine
    batch = oracle_lib.generate(48, seed=616, n_clients=8, ops_per_doc=500, max_lag=16, n_keys=2, n_values=15,
                                p_insert=0.5, p_remove=0.35, p_overlap=0.3, p_null=0.2, p_rewrite=0.1,
                                p_insert_props=0.6, p_marker=0.5)
    o = oracle_lib.Oracle(batch.n_docs).apply(batch)
    eng = MergeEngine(batch.n_docs, ops_per_launch=32)
    eng.set_label_keys(0, 1)  # (tile labels on key 0, range labels on key 1)
    eng.apply(batch)
    masks = [label_mask(k) for k in range(4)]
    q, want = [], []
    for d in range(batch.n_docs):
        for pos in range(0, eng.length(d) + 2):
            for lab in range(4):
                q.append((d, pos, RANGE_KEY, 0, 0, 0, masks[lab].view('<u4'), 0))
                want.append(o.stack_context(d, pos, RANGE_KEY, masks[lab]))
    got = eng.range_stacks(np.array(q, dtype=TILE_QUERY_DTYPE))
    assert sum(1 for w in want if w) > 1000
    gl = _as_lists(got)
    bad = [i for i in range(len(want)) if gl[i] != want[i]]
    assert not bad, [(q[i][:3], gl[i], want[i]) for i in bad[:5]]
    assert all(len(s) == 0 or (s['ordinal'] >= 0).all() for s in got)


@pytest.mark.gpu
def test_range_stacks_rejects_a_bad_document():
    """argument checks happen on the host, before any device work"""
    from fluidframework_amd.engine import TILE_QUERY_DTYPE, MergeEngine, MtError
    eng = MergeEngine(2)
    with pytest.raises(MtError):
        eng.range_stacks(np.array([(5, 0, RANGE_KEY, 0, 0, 0, np.zeros(8, '<u4'), 0)], dtype=TILE_QUERY_DTYPE))
