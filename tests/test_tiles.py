"""findTile (tiles): Client.findTile(startPos, label, preceding)
(client.ts:1073-1076 -> mergeTree.ts:1763-1789) for the own client, pinned by the reference itself:
tests/golden/tiles.expected.jsonl holds the answers the reference's observer Client gave on the
tiles_* logs (tests/golden/make_tiles.py) -- the client.spec.ts findTile cases restated as remote
ops, marker-heavy synthetic logs, and tiles_annot: label annotates that leave the reference's
HierMergeBlock caches stale (146 of its 2,176 answers differ from an answer from the current labels).  Labels ride on property key 0 (value id v = the labels L<i>
of its bits i, js/mtlog.js tileLabels); a query's label becomes the set of value ids whose label
arrays hold it (`label_mask`).  The oracle restates search / backwardSearch over its pointer tree;
the engine answers a batch of queries on the device (mt_find_tiles)."""
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN

TILE_KEY = 0
LOGS = ['tiles_scenarios', 'tiles_synth', 'tiles_annot']


def label_mask(label):
    """256-bit mask (32 bytes) of the value ids whose label arrays contain L<label>"""
    m = np.zeros(32, dtype=np.uint8)
    for v in range(1, 256):
        if (v >> label) & 1:
            m[v >> 3] |= 1 << (v & 7)
    return m


def load_tiles():
    out = {}
    with open(os.path.join(GOLDEN, 'tiles.expected.jsonl')) as f:
        for line in f:
            r = json.loads(line)
            out.setdefault(r['log'], []).append(r)
    return out


def test_fixture_covers_both_directions_and_misses():
    rows = [r for v in load_tiles().values() for r in v]
    ans = [a for r in rows for a in r['answers']]
    assert {a[2] for a in ans} == {0, 1}
    assert any(a[3] is None for a in ans) and sum(a[3] is not None for a in ans) > 500
    assert all(r['err'] is None for r in rows)


@pytest.mark.parametrize('name', LOGS)
def test_oracle_find_tile_matches_reference(oracle_lib, name):
    from fluidframework_amd.oplog import OpBatch
    batch = OpBatch.load(os.path.join(GOLDEN, name + '.mtlog'))
    o = oracle_lib.Oracle(batch.n_docs).apply(batch)
    masks = [label_mask(k) for k in range(4)]
    for r in load_tiles()[name]:
        for pos, lab, prec, want in r['answers']:
            got = o.find_tile(r['doc'], pos, TILE_KEY, masks[lab], bool(prec))
            assert got == want, (name, r['doc'], pos, lab, prec)


def _queries(rows, masks):
    from fluidframework_amd.engine import TILE_QUERY_DTYPE
    q = []
    for r in rows:
        for pos, lab, prec, _ in r['answers']:
            q.append((r['doc'], pos, TILE_KEY, prec, 0, 0, masks[lab].view('<u4'), 0))
    return np.array(q, dtype=TILE_QUERY_DTYPE)


@pytest.mark.gpu
@pytest.mark.parametrize('name', LOGS)
def test_engine_find_tiles_match_reference(name):
    from fluidframework_amd.engine import MergeEngine
    from fluidframework_amd.oplog import OpBatch
    batch = OpBatch.load(os.path.join(GOLDEN, name + '.mtlog'))
    eng = MergeEngine(batch.n_docs, ops_per_launch=16)
    eng.set_label_keys(0, 1)  # (tile labels on key 0, range labels on key 1)
    eng.apply(batch)
    rows = load_tiles()[name]
    masks = [label_mask(k) for k in range(4)]
    got = eng.find_tiles(_queries(rows, masks))
    want = [a[3] for r in rows for a in r['answers']]
    for i, (g, w) in enumerate(zip(got['pos'], want)):
        assert (None if g < 0 else int(g)) == w, (name, i)


@pytest.mark.gpu
def test_engine_find_tiles_match_oracle_on_fuzz(oracle_lib):
    """Marker-heavy fuzz (with zamboni, so empty leaf blocks and removed tiles occur): every
    position of every document, every label, both directions."""
    from fluidframework_amd.engine import MergeEngine, TILE_QUERY_DTYPE
    batch = oracle_lib.generate(48, seed=515, n_clients=8, ops_per_doc=500, max_lag=16, n_keys=2, n_values=15,
                                p_insert=0.5, p_remove=0.35, p_overlap=0.3, p_null=0.2, p_rewrite=0.1,
                                p_insert_props=0.6, p_marker=0.4)
    o = oracle_lib.Oracle(batch.n_docs).apply(batch)
    eng = MergeEngine(batch.n_docs, ops_per_launch=32)
    eng.set_label_keys(0, 1)  # (tile labels on key 0, range labels on key 1)
    eng.apply(batch)
    masks = [label_mask(k) for k in range(4)]
    q, want = [], []
    for d in range(batch.n_docs):
        n = eng.length(d)
        for pos in range(0, n + 2):
            for lab in range(4):
                for prec in (0, 1):
                    q.append((d, pos, TILE_KEY, prec, 0, 0, masks[lab].view('<u4'), 0))
                    want.append(o.find_tile(d, pos, TILE_KEY, masks[lab], bool(prec)))
    got = eng.find_tiles(np.array(q, dtype=TILE_QUERY_DTYPE))
    assert len(got) == len(want)
    bad = [i for i, (g, w) in enumerate(zip(got['pos'], want)) if (None if g < 0 else int(g)) != w]
    assert not bad, [(q[i][:4], int(got['pos'][i]), want[i]) for i in bad[:5]]
