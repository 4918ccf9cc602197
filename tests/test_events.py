"""Delta / maintenance events: what Client.mergeTreeDeltaCallback and
mergeTreeMaintenanceCallback receive (mergeTreeDeltaCallback.ts:15-73), fired inside applyMsg at
mergeTree.ts:1981-1988 (INSERT), 2705-2712 (REMOVE), 2592-2600 (ANNOTATE, propertyDeltas),
2231-2236 (SPLIT), 1335-1340 (APPEND), 1310-1315 (UNLINK).

Pinned by the reference itself: tests/golden/events.jsonl holds the callbacks the reference's own
observer Client fired on the golden logs (tests/golden/make_events.py; canonical form in
fluidframework_amd/events.py) -- in full for the scenario / marker / error / empty-insert logs, as a
count + SHA-256 per document for the synthetic ones.  The oracle must reproduce them exactly, and
the engine (every capacity class on the LDS engine while recording) must reproduce the oracle's.
"""
import hashlib
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN, load_golden

LOGS = ['scenarios', 'markers', 'errors', 'empty_inserts', 'synth_tiny', 'synth_c3', 'synth_c4', 'synth_markers', 'wide',
        'wide_synth']


def _golden_events():
    out = {}
    with open(os.path.join(GOLDEN, 'events.jsonl')) as f:
        for line in f:
            r = json.loads(line)
            out.setdefault(r['log'], {})[r['doc']] = r
    return out


def _err_seqs(name):
    _, exp = load_golden(name)
    return {r['doc']: r['err_seq'] for r in exp if r.get('err') is not None}


def _matches(rec, events, err_seq):
    """events of one document vs its golden record; a document the reference threw on keeps the
    callbacks of the messages before the failing seq (the engine halts before that message)"""
    if err_seq is not None:
        events = [e for e in events if e[0] < err_seq]
    if 'events' in rec:
        return events == rec['events']
    return len(events) == rec['n'] and hashlib.sha256(
        json.dumps(events, separators=(',', ':')).encode()).hexdigest() == rec['sha256']


def test_golden_events_cover_every_callback_kind():
    gold = _golden_events()
    ops = set()
    for name in ('scenarios', 'markers', 'errors', 'empty_inserts'):
        for rec in gold[name].values():
            for e in rec['events']:
                ops.add(e[1])
                if e[1] in (1, 2) and not e[2]:
                    ops.add('empty')
                if e[1] == 0 and e[2] and e[2][0][0] == -1:
                    ops.add('unlinked insert')
    assert ops >= {0, 1, 2, -1, -2, -3, 'empty', 'unlinked insert'}, ops
    assert sum(r['n'] for r in gold['synth_c4'].values()) > 10000


def test_callbacks_grouping():
    from fluidframework_amd.events import EVENT_DTYPE, EVF_EMPTY, EVF_FIRST, callbacks
    rows = np.zeros(6, dtype=EVENT_DTYPE)
    z = [0] * 32
    # (seq, op, flags, pad, leaf, pos, len, pmask, pvals, pad2)
    rows[0] = (7, -2, EVF_FIRST, 0, 3, -1, 2, 0, z, 0)
    rows[1] = (7, -2, 0, 0, 4, -1, 5, 0, z, 0)
    rows[2] = (7, 1, EVF_FIRST | EVF_EMPTY, 0, -1, -1, 0, 0, z, 0)
    rows[3] = (8, 2, EVF_FIRST, 0, 2, 9, 1, 0b101, [0, 3, 0] + [0] * 29, 0)  # k0, k2 -> null (k1 unmasked)
    rows[4] = (8, 2, 0, 0, 3, 10, 4, 0b10, [0, 9] + [0] * 30, 0)
    rows[5] = (8, 2, 0, 0, 4, 14, 1, (1 << 12) | (1 << 27), [0] * 12 + [40000] + [0] * 14 + [5, 0, 0, 0, 0], 0)
    cb = callbacks(rows)
    assert cb == [[7, -2, [[3, -1, 2, None], [4, -1, 5, None]]], [7, 1, []],
                  [8, 2, [[2, 9, 1, {'k0': None, 'k2': None}], [3, 10, 4, {'k1': 9}], [4, 14, 1, {'k12': 40000, 'k27': 5}]]]]


@pytest.mark.parametrize('name', LOGS)
def test_oracle_events_match_reference(oracle_lib, name):
    gold = _golden_events()[name]
    errs = _err_seqs(name)
    batch, _ = load_golden(name)
    o = oracle_lib.Oracle(batch.n_docs).record_events().apply(batch)
    for d in range(batch.n_docs):
        assert _matches(gold[d], o.events(d), errs.get(d)), (name, d)


def _engine(n, b, **kw):
    from fluidframework_amd.engine import MergeEngine
    return MergeEngine(n, ops_per_launch=b, **kw)


@pytest.mark.gpu
@pytest.mark.parametrize('b', [0, 3])
def test_engine_events_match_reference(b):
    gold = _golden_events()
    for name in LOGS:
        errs = _err_seqs(name)
        batch, exp = load_golden(name)
        eng = _engine(batch.n_docs, b).enable_events(1 << 16)
        eng.apply(batch)
        got = eng.drain_events()
        cs = eng.checksums()
        for d in range(batch.n_docs):
            assert _matches(gold[name][d], got[d], errs.get(d)), (name, d, b)
            assert '%016x' % cs[d] == exp[d]['checksum'], (name, d, b)
        eng.close()


@pytest.mark.gpu
def test_engine_events_match_oracle_across_drains(oracle_lib):
    """A fuzz log in two halves with a drain between them, at b = 8: every callback of every
    document, in order, equal to the oracle's; the second drain returns only the second half's."""
    from fluidframework_amd.oplog import OpBatch
    full = oracle_lib.generate(96, seed=77, n_clients=24, ops_per_doc=600, max_lag=48, n_keys=4, n_values=6,
                               p_insert=0.45, p_remove=0.35, p_overlap=0.5, p_null=0.1, p_rewrite=0.05,
                               p_insert_props=0.2, p_marker=0.1)
    halves = []
    for lo, hi in ((0, 300), (300, 600)):
        rows = [np.arange(int(full.row_ptr[d]) + lo, int(full.row_ptr[d]) + hi) for d in range(full.n_docs)]
        idx = np.concatenate(rows)
        halves.append(OpBatch(full.ops[idx].copy(), full.payload,
                              np.arange(0, full.n_docs * (hi - lo) + 1, hi - lo, dtype=np.uint32)))
    o = oracle_lib.Oracle(full.n_docs).record_events().apply(full)
    eng = _engine(full.n_docs, 8).enable_events(1 << 15)
    got = []
    for h in halves:
        eng.apply(h)
        got.append(eng.drain_events())
    split_seq = [int(full.ops[int(full.row_ptr[d]) + 300]['seq']) for d in range(full.n_docs)]
    for d in range(full.n_docs):
        want = o.events(d)
        assert eng.error(d) == (0, 0), d
        assert got[0][d] == [e for e in want if e[0] < split_seq[d]], d
        assert got[1][d] == [e for e in want if e[0] >= split_seq[d]], d
    assert np.array_equal(eng.checksums(), o.checksums())


@pytest.mark.gpu
def test_engine_events_overflow_halts_the_document(oracle_lib):
    """A document whose callbacks outgrow its buffer halts with MT_DERR_EVENTS (8); the records it
    kept are the first ones the oracle fired, and its neighbours are unaffected."""
    batch = oracle_lib.generate(8, seed=3, n_clients=6, ops_per_doc=200, max_lag=8, n_keys=2, n_values=4,
                                p_insert=0.6, p_remove=0.3)
    o = oracle_lib.Oracle(batch.n_docs).record_events().apply(batch)
    counts = [len(o.event_rows(d)) for d in range(batch.n_docs)]
    cap = sorted(counts)[len(counts) // 2]  # about half of the documents overflow
    eng = _engine(batch.n_docs, 16).enable_events(cap)
    eng.apply(batch)
    rows, rp = eng.drain_event_rows()
    want = o.checksums()
    got = eng.checksums()
    for d in range(batch.n_docs):
        mine = rows[rp[d]:rp[d + 1]]
        ref = o.event_rows(d)
        assert np.array_equal(mine, ref[:len(mine)]), d
        if counts[d] > cap:
            assert eng.error(d)[0] == 8, d
            assert len(mine) == cap
        else:
            assert eng.error(d) == (0, 0) and got[d] == want[d], d


@pytest.mark.gpu
def test_engine_events_large_document(oracle_lib):
    """A document past 2048 segments (the HBM-workspace form of the LDS engine) records the same
    callbacks as the oracle."""
    from fluidframework_amd.oplog import INSERT, NOOP, OP_DTYPE, REMOVE, OpBatch
    recs, payload = [], bytearray()
    for k in range(2600):
        recs.append((k + 1, k, 0, 1 + k % 3, INSERT, 0, k % 17, 0, len(payload), 1))
        payload += b'abcdefghij'[k % 10:k % 10 + 1]
    recs.append((2601, 2600, 0, 2, REMOVE, 0, 100, 900, 0, 0))
    recs.append((2602, 2601, 2601, 1, NOOP, 0, 0, 0, 0, 0))
    batch = OpBatch(np.array(recs, dtype=OP_DTYPE), np.frombuffer(bytes(payload), np.uint8),
                    np.array([0, len(recs)], np.uint32))
    o = oracle_lib.Oracle(1).record_events().apply(batch)
    eng = _engine(1, 64, seg_capacity=4096).enable_events(1 << 16)
    eng.apply(batch)
    assert eng.error(0) == (0, 0)
    assert eng.drain_events()[0] == o.events(0)
    assert eng.checksums()[0] == o.checksums()[0]


@pytest.mark.gpu
def test_engine_events_switch_on_and_off(oracle_lib):
    """Recording can start after the register engine has applied part of the log and stop again:
    the first third unrecorded (register engine), the second recorded (LDS engine), the last
    unrecorded; the recorded callbacks are the oracle's for exactly the middle third, and the final
    state is the oracle's."""
    from fluidframework_amd.oplog import OpBatch
    full = oracle_lib.generate(64, seed=91, n_clients=16, ops_per_doc=480, max_lag=32, n_keys=3, n_values=5,
                               p_insert=0.5, p_remove=0.3, p_overlap=0.5, p_null=0.1, p_insert_props=0.2)
    parts = []
    for lo, hi in ((0, 160), (160, 320), (320, 480)):
        idx = np.concatenate([np.arange(int(full.row_ptr[d]) + lo, int(full.row_ptr[d]) + hi)
                              for d in range(full.n_docs)])
        parts.append(OpBatch(full.ops[idx].copy(), full.payload,
                             np.arange(0, full.n_docs * (hi - lo) + 1, hi - lo, dtype=np.uint32)))
    o = oracle_lib.Oracle(full.n_docs).record_events().apply(full)
    eng = _engine(full.n_docs, 32)
    eng.apply(parts[0])
    eng.enable_events(1 << 14)
    eng.apply(parts[1])
    got = eng.drain_events()
    eng.enable_events(0)
    eng.apply(parts[2])
    for d in range(full.n_docs):
        a = int(full.ops[int(full.row_ptr[d]) + 160]['seq'])
        b = int(full.ops[int(full.row_ptr[d]) + 320]['seq'])
        assert got[d] == [e for e in o.events(d) if a <= e[0] < b], d
    assert np.array_equal(eng.checksums(), o.checksums())
