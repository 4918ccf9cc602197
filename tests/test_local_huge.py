"""An editing client beyond the editing form's LDS limits: documents past 1024 segments
(MT_LOC_CAP) and more than 64 pending edits -- the editing form's HBM-workspace forms (mt_apply.hip
apply_kernel_g<CAP, false, true, GW>, mt_launch_apply_loc_big; include/mtgpu.h MT_SEQ_LOCAL).

Pinned by the reference itself: tests/golden/<log>.expected.jsonl holds the canonical states of a
reference Client c1 replaying <log>.mtlog (tests/golden/make_local_huge.py: the local_farm.js farm
of reference clients, 4 clients, c1 lagging), at checkpoints and at the end:
  * local_huge: 32000 edits; both documents pass 1024 segments (up to 1609) with edits pending;
  * local_offline: c1 goes offline for 12-24 rounds now and then, so 110-170 of its edits are
    pending at once (acked in order when it comes back);
  * local_offline_long: c1 stays offline for 90-120 rounds, so 400-484 of its edits are pending at once
    (the form's 512 pending-edit slots), and its documents pass 1024 segments meanwhile."""
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN
from test_local import checkpoint_batch, prefix

NAME = 'local_huge'
OFFLINE = 'local_offline'
OFFLINE_LONG = 'local_offline_long'


def load_rows(name=NAME):
    with open(os.path.join(GOLDEN, name + '.expected.jsonl')) as f:
        return [json.loads(line) for line in f]


def max_pending(batch, doc):
    """the most edits of the document's editing client pending at once (local edits not yet acked)"""
    a, b = int(batch.row_ptr[doc]), int(batch.row_ptr[doc + 1])
    ops = batch.ops[a:b]
    local = ops['seq'] == -1
    ack = (ops['seq'] > 0) & (ops['client'] == 1) & ((ops['flags'] & 4) == 0)  # (a GROUP acks once)
    return int(np.max(np.cumsum(local.astype(np.int64) - ack.astype(np.int64))))


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


def test_offline_fixture_has_more_than_64_pending_edits():
    from fluidframework_amd.oplog import OpBatch
    b = OpBatch.load(os.path.join(GOLDEN, OFFLINE + '.mtlog'))
    rows = load_rows(OFFLINE)
    assert all(r['err'] is None for r in rows)
    pend = [max_pending(b, d) for d in range(b.n_docs)]
    assert min(pend) > 100, pend


def test_long_offline_fixture_has_400_pending_edits():
    from fluidframework_amd.oplog import OpBatch
    b = OpBatch.load(os.path.join(GOLDEN, OFFLINE_LONG + '.mtlog'))
    rows = load_rows(OFFLINE_LONG)
    assert all(r['err'] is None for r in rows)
    pend = [max_pending(b, d) for d in range(b.n_docs)]
    assert min(pend) > 400 and max(pend) <= 512, pend


@pytest.mark.parametrize('name', [NAME, OFFLINE, OFFLINE_LONG])
def test_oracle_editing_client_matches_reference_beyond_lds_limits(oracle_lib, name):
    from fluidframework_amd.oplog import OpBatch
    batch = OpBatch.load(os.path.join(GOLDEN, name + '.mtlog'))
    o = oracle_lib.Oracle(batch.n_docs).apply(batch)
    for r in load_rows(name):
        d = r['doc']
        assert o.error(d) == (0, 0), (d, o.error(d))
        assert o.state(d) == r['states'][-1][1], d
        for k, want in r['states'][-3:-1]:
            assert oracle_lib.Oracle(1).apply(prefix(batch, d, k)).state(0) == want, (d, k)


@pytest.mark.parametrize('name', [OFFLINE, OFFLINE_LONG])
def test_oracle_events_past_64_pending_edits_match_reference(oracle_lib, name):
    import hashlib
    from fluidframework_amd.oplog import OpBatch
    batch = OpBatch.load(os.path.join(GOLDEN, name + '.mtlog'))
    o = oracle_lib.Oracle(batch.n_docs).record_events().apply(batch)
    with open(os.path.join(GOLDEN, name + '.events.jsonl')) as f:
        gold = [json.loads(x) for x in f]
    for g in gold:
        ev = o.events(g['doc'])
        assert len(ev) == g['n'] and hashlib.sha256(json.dumps(ev, separators=(',', ':')).encode()).hexdigest() == \
            g['sha256'], g['doc']


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
            assert eng.class_kernel(editing_g) == 'mt::apply_kernel_g<2048, false, true, 1>'
        eng.close()


@pytest.mark.gpu
@pytest.mark.parametrize('name,b', [(OFFLINE, 1), (OFFLINE, 32), (OFFLINE_LONG, 1), (OFFLINE_LONG, 32)])
def test_engine_editing_form_past_64_pending_edits_matches_reference(name, b):
    """110-170 pending edits at once: every checkpoint state and the final state equal the
    reference's; the documents ran on the form with 512 pending-edit slots (class stats
    MT_CLASS_EDITING | MT_CLASS_GROUPS | 1024, mt::apply_kernel_g<1024, false, true, 8>), which they
    enter with edits pending (their group masks and stamps re-laid) and keep for good."""
    from fluidframework_amd.engine import MergeEngine
    from fluidframework_amd.oplog import OpBatch
    batch = OpBatch.load(os.path.join(GOLDEN, name + '.mtlog'))
    rows = load_rows(name)
    groups = 0x40000000 | 0x08000000 | 1024
    for q in range(len(rows[0]['states'])):
        cb = checkpoint_batch(batch, rows, q)
        eng = MergeEngine(cb.n_docs, ops_per_launch=b)
        eng.apply(cb)
        used = {cap: n for cap, _, n, _ in eng.last_class_stats() if n}
        for i, r in enumerate(rows):
            assert eng.error(i) == (0, 0), (r['doc'], q, eng.error(i))
            assert eng.state(i) == r['states'][q][1], (r['doc'], q, b)
        if name == OFFLINE and max(max_pending(cb, i) for i in range(cb.n_docs)) > 64:
            assert used.get(groups, 0) > 0, used
        if name == OFFLINE_LONG and max(max_pending(cb, i) for i in range(cb.n_docs)) > 64:
            assert any(cap & 0x08000000 for cap in used), used  # (at 1024 or, past 1024 segments, 4096 slots)
            assert eng.class_kernel(groups) == 'mt::apply_kernel_g<1024, false, true, 8>'
        eng.close()


@pytest.mark.gpu
@pytest.mark.parametrize('name', [OFFLINE, OFFLINE_LONG])
def test_engine_editing_form_past_64_pending_edits_events_match_reference(name):
    """The delta callbacks the wide-group form records (mt_events_enable) equal the reference
    client's (tests/golden/<name>.events.jsonl: count + SHA-256 per document)."""
    import hashlib
    from fluidframework_amd.engine import MergeEngine
    from fluidframework_amd.oplog import OpBatch
    batch = OpBatch.load(os.path.join(GOLDEN, name + '.mtlog'))
    eng = MergeEngine(batch.n_docs, ops_per_launch=16).enable_events(1 << 16)
    eng.apply(batch)
    got = eng.drain_events()
    with open(os.path.join(GOLDEN, name + '.events.jsonl')) as f:
        gold = [json.loads(x) for x in f]
    for g in gold:
        d = g['doc']
        assert eng.error(d) == (0, 0), (d, eng.error(d))
        ev = got[d]
        assert len(ev) == g['n'] and hashlib.sha256(json.dumps(ev, separators=(',', ':')).encode()).hexdigest() == \
            g['sha256'], d
    eng.close()


@pytest.mark.gpu
def test_editing_pool_rows_scale_with_the_documents_that_need_them():
    """Two of 100,000 documents pass 1024 editing segments: only they get rows of the editing form's
    big pool (mt_state.h locbig, MT_LOC_BIGCAP slots), so the engine's device memory grows by far
    less than 100 MB (a re-lay of every document's editing rows at 4096 slots would take ~11 GB),
    and both end in the reference's final states."""
    import ctypes
    from fluidframework_amd.engine import MergeEngine
    from fluidframework_amd.hipmem import hip
    from fluidframework_amd.oplog import OpBatch
    src = OpBatch.load(os.path.join(GOLDEN, NAME + '.mtlog'))
    rows = load_rows()
    D = 100_000
    place = {r['doc']: D // 2 + i * (D // 2 - 1) for i, r in enumerate(rows)}  # docs 50000 and 99999
    cnt = np.zeros(D, dtype=np.int64)
    idx = []
    for d in sorted(place, key=place.get):
        a, b = int(src.row_ptr[d]), int(src.row_ptr[d + 1])
        idx.append(np.arange(a, b))
        cnt[place[d]] = b - a
    rp = np.concatenate([[0], np.cumsum(cnt)]).astype(np.uint32)
    batch = OpBatch(src.ops[np.concatenate(idx)].copy(), src.payload, rp)

    def free_bytes():
        f, t = ctypes.c_size_t(), ctypes.c_size_t()
        assert hip().hipMemGetInfo(ctypes.byref(f), ctypes.byref(t)) == 0
        return f.value

    eng = MergeEngine(D, ops_per_launch=32)
    before = free_bytes()
    eng.apply(batch)
    grown = before - free_bytes()
    used = {cap: n for cap, _, n, _ in eng.last_class_stats() if n}
    for r in rows:
        k = place[r['doc']]
        assert eng.error(k) == (0, 0), (r['doc'], eng.error(k))
        assert eng.state(k) == r['states'][-1][1], r['doc']
    assert used.get(0x40000000 | 2048, 0) > 0, used
    assert grown < 100 << 20, f'device memory grew by {grown >> 20} MiB'
    eng.close()


def _editing_grow_batch(n_local):
    """One editing document that grows past 4096 segments: client 1's local inserts (seq -1), each
    acked by its sequenced echo at once, and every tenth a remote insert by client 2; the msn stays
    0 (no zamboni), and each insert carries its own property value, so segments never merge."""
    from fluidframework_amd.oplog import F_PROPS, INSERT, OP_DTYPE, OpBatch
    recs, payload = [], bytearray()

    def rec(seq, ref, client, pos, data):
        recs.append((seq, ref, 0, client, INSERT, F_PROPS | (1 << 3), pos, 0, len(payload), len(data)))
        payload.extend(data)
    s = length = 0
    for i in range(n_local):
        pos = (i * 7919) % (length + 1)
        data = b'ab'[i % 2:i % 2 + 1] + bytes([0, 1 + i % 250])
        rec(-1, s, 1, pos, data)     # the local edit (MT_SEQ_LOCAL) ...
        rec(s + 1, s, 1, pos, data)  # ... and its ack
        s += 1
        length += 1
        if i % 10 == 9:
            rec(s + 1, s, 2, (i * 31) % (length + 1), b'z' + bytes([1, 1 + i % 200]))
            s += 1
            length += 1
    return OpBatch(np.array(recs, dtype=OP_DTYPE), np.frombuffer(bytes(payload), np.uint8),
                   np.array([0, len(recs)], dtype=np.uint32))


def test_oracle_editing_document_grows_past_4096_segments(oracle_lib):
    b = _editing_grow_batch(4500)
    o = oracle_lib.Oracle(1).apply(b)
    assert o.error(0) == (0, 0) and 4096 < o.nsegs(0) < 8192, o.nsegs(0)


@pytest.mark.gpu
def test_engine_editing_form_past_4096_segments():
    """The editing form's 8192-slot HBM-workspace class (apply_kernel_g<8192, false, true, 1>, a big-pool
    row of MT_LOC_BIGCAP = 8192 slots): the device ends in the oracle's state."""
    import oracle.oracle as oracle_lib
    from fluidframework_amd.engine import MergeEngine
    b = _editing_grow_batch(4500)
    o = oracle_lib.Oracle(1).apply(b)
    eng = MergeEngine(1, seg_capacity=8192, ops_per_launch=32)
    eng.apply(b)
    assert eng.error(0) == (0, 0), eng.error(0)
    assert eng.state(0) == o.state(0)
    assert eng.class_kernel(0x40000000 | 8192) == 'mt::apply_kernel_g<8192, false, true, 1>'
    eng.close()
