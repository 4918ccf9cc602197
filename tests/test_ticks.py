"""The tick-major feed's host layout (mt_log_to_ticks, include/mtgpu.h "tick-major feed"): no device
work, so it runs on the CPU.  Laying a document-major op log out tick-major and reading every
document back tick by tick must give each document's records (and payload bytes) in their order,
with each raw message still carrying its own record; the apply of the ticks is pinned on the GPU
(tests/test_gpu_parity.py::test_tick_feed_equals_reference, test_gpu_deli.py)."""
import numpy as np
import pytest

from conftest import load_golden


def _doc_records(log, d):
    """Document d's records, read back tick by tick: (records with absolute payload, payload bytes)."""
    recs, pays = [], []
    D = log.n_docs
    for t in range(log.n_ticks):
        rp = log.row_ptrs[t * (D + 1):(t + 1) * (D + 1)]
        o0, p0 = int(log.tick_ops[t]), int(log.tick_payload[t])
        for i in range(int(rp[d]), int(rp[d + 1])):
            r = log.ops[o0 + i]
            recs.append(r)
            off = p0 + int(r['payload_off'])
            pays.append(bytes(log.payload[off:off + int(r['payload_len'])]))
    return recs, pays


def _tick_span(t, per, first):
    """[lo, hi) of a document's records in tick t (mt_log_to_ticks_ramp: tick u holds min(per, first << u))."""
    lo = 0
    for u in range(t):
        lo += min(per, first << u)
    return lo, lo + min(per, first << t)


def _n_ticks(mx, per, first):
    t = c = 0
    while c < mx:
        c += min(per, first << t)
        t += 1
    return max(1, t)


def _check_layout(batch, log, per, first=None):
    from fluidframework_amd.oplog import OP_DTYPE
    first = per if first is None else first
    lens = np.diff(batch.row_ptr.astype(np.int64))
    assert log.n_ticks == _n_ticks(int(lens.max()), per, first)
    assert int(log.tick_ops[-1]) == batch.n_ops
    used = int(batch.ops['payload_len'].astype(np.int64).sum())
    assert int(log.tick_payload[-1]) == used  # compacted: no unused payload bytes travel
    for d in range(batch.n_docs):
        recs, pays = _doc_records(log, d)
        src = batch.ops[batch.row_ptr[d]:batch.row_ptr[d + 1]]
        assert len(recs) == len(src)
        for k, (r, p) in enumerate(zip(recs, pays)):
            s = src[k]
            for f in OP_DTYPE.names:
                if f != 'payload_off':
                    assert r[f] == s[f], (d, k, f)
            off = int(s['payload_off'])
            assert p == bytes(batch.payload[off:off + int(s['payload_len'])])
        # tick t holds records [t*per, (t+1)*per) of the document (tick 0: [0, first))
        for t in range(log.n_ticks):
            rp = log.row_ptrs[t * (batch.n_docs + 1):(t + 1) * (batch.n_docs + 1)]
            lo, hi = _tick_span(t, per, first)
            assert int(rp[d + 1] - rp[d]) == max(0, min(hi, len(src)) - lo)


@pytest.mark.parametrize('per', [1, 5, 32, 4096])
def test_layout_of_golden_logs(per):
    from fluidframework_amd.ticks import TickLog
    batch, _ = load_golden('synth_c3')
    log = TickLog.from_batch(batch, per, pinned=False)
    _check_layout(batch, log, per)


@pytest.mark.parametrize('per,first', [(32, 8), (32, 1), (5, 4), (4096, 100), (32, 3), (1000, 1)])
def test_ramp_layout_of_golden_logs(per, first):
    """A ramp of short first ticks (mt_log_to_ticks_ramp): the same records in the same order, tick t
    cut to min(per, first << t) records per document."""
    from fluidframework_amd.ticks import TickLog
    batch, _ = load_golden('synth_c3')
    log = TickLog.from_batch(batch, per, pinned=False, first=first)
    _check_layout(batch, log, per, first)


def test_ramp_first_tick_is_checked():
    from fluidframework_amd.engine import MtError
    from fluidframework_amd.ticks import TickLog
    batch, _ = load_golden('synth_c2')
    for first in (0, 33):
        with pytest.raises(MtError):
            TickLog.from_batch(batch, 32, pinned=False, first=first)


def test_layout_of_ragged_documents():
    """Documents of very different lengths (some empty) and payload offsets out of record order."""
    from fluidframework_amd.oplog import OP_DTYPE, OpBatch
    from fluidframework_amd.ticks import TickLog
    rng = np.random.default_rng(7)
    lens = rng.integers(0, 90, size=37)
    lens[[3, 11]] = 0
    n = int(lens.sum())
    ops = np.zeros(n, dtype=OP_DTYPE)
    ops['seq'] = np.arange(n) + 1
    ops['payload_len'] = rng.integers(0, 20, size=n)
    total = int(ops['payload_len'].sum())
    perm = rng.permutation(n)  # payload blocks stored in a shuffled order, with gaps
    offs = np.zeros(n, dtype=np.int64)
    cur = 0
    for i in perm:
        offs[i] = cur
        cur += int(ops['payload_len'][i]) + int(rng.integers(0, 3))
    ops['payload_off'] = offs
    payload = rng.integers(0, 256, size=cur + 1).astype(np.uint8)
    row_ptr = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint32)
    batch = OpBatch(ops, payload, row_ptr)
    for per, first in ((1, 1), (7, 7), (32, 32), (200, 200), (32, 3), (7, 1)):
        log = TickLog.from_batch(batch, per, pinned=False, first=first)
        _check_layout(batch, log, per, first)
        assert int(log.tick_payload[-1]) == total


def test_raw_messages_follow_their_records():
    """C5-shaped raw streams (joins, then one message per record, plus no-ops between): every message
    lands in its record's tick (messages without one: the tick of the document's previous record)
    with op_index rebased to the record's index in that tick, and each document's messages keep
    their order across ticks."""
    from fluidframework_amd.deli import JOIN, NOOP, OP, RAW_DTYPE
    from fluidframework_amd.ticks import TickLog
    batch, _ = load_golden('synth_c2')
    D = batch.n_docs
    rng = np.random.default_rng(3)
    msgs, mrp = [], [0]
    for d in range(D):
        m = [(0, 0, c, JOIN, 0) for c in range(1, 9)]
        for i in range(int(batch.row_ptr[d]), int(batch.row_ptr[d + 1])):
            m.append((i, 0, 1, OP, i + 1))
            if rng.random() < 0.05:
                m.append((0, 0, 2, NOOP, 0))
        msgs += m
        mrp.append(mrp[-1] + len(m))
    raw = np.zeros(len(msgs), dtype=RAW_DTYPE)
    for k, f in enumerate(('csn', 'ref_seq', 'client', 'kind', 'op_index')):
        raw[f] = [x[k] for x in msgs]
    mrp = np.array(mrp, dtype=np.uint32)
    for per, first in ((16, 16), (16, 5)):
        log = TickLog.from_batch(batch, per, msgs=raw, msg_row_ptr=mrp, pinned=False, first=first)
        _check_messages(batch, log, raw, mrp)


def _check_messages(batch, log, raw, mrp):
    from fluidframework_amd.deli import RAW_DTYPE
    D = batch.n_docs
    assert int(log.tick_msgs[-1]) == len(raw)
    for d in range(D):
        got = []
        for t in range(log.n_ticks):
            rp = log.msg_row_ptrs[t * (D + 1):(t + 1) * (D + 1)]
            orp = log.row_ptrs[t * (D + 1):(t + 1) * (D + 1)]
            m0 = int(log.tick_msgs[t])
            for j in range(int(rp[d]), int(rp[d + 1])):
                x = log.msgs[m0 + j].copy()
                if x['op_index']:
                    k = int(x['op_index']) - 1
                    assert orp[d] <= k < orp[d + 1]  # a record of this document in this tick
                    r, s = log.ops[int(log.tick_ops[t]) + k], batch.ops[int(x['csn'])]  # (csn: the batch index)
                    assert (r['seq'], r['pos1'], r['pos2'], r['type']) == (s['seq'], s['pos1'], s['pos2'], s['type'])
                    x['op_index'] = int(x['csn']) + 1
                got.append(x)
        want = raw[mrp[d]:mrp[d + 1]]
        assert np.array_equal(np.array(got, dtype=RAW_DTYPE), want)


def test_malformed_logs_are_refused():
    from fluidframework_amd.engine import MtError
    from fluidframework_amd.oplog import OpBatch
    from fluidframework_amd.ticks import TickLog
    batch, _ = load_golden('synth_c2')
    bad = OpBatch(batch.ops.copy(), batch.payload, batch.row_ptr)
    bad.ops['payload_off'][5] = len(batch.payload)  # past the payload
    bad.ops['payload_len'][5] = 1
    with pytest.raises(MtError):
        TickLog.from_batch(bad, 32, pinned=False)
    rp = batch.row_ptr.copy()
    rp[2], rp[3] = rp[3], rp[2]  # not monotone
    with pytest.raises(MtError):
        TickLog.from_batch(OpBatch(batch.ops, batch.payload, rp), 32, pinned=False)


def test_messages_out_of_record_order_are_refused():
    """A document's messages must carry its records in stream order, each once: a message pointing at a
    record before the previous message's would land in an earlier tick than that message and deli
    would ticket the stream out of order, so the layout refuses it (MT_ERR_ARG)."""
    from fluidframework_amd.deli import OP, RAW_DTYPE
    from fluidframework_amd.engine import MtError
    from fluidframework_amd.ticks import TickLog
    batch, _ = load_golden('synth_c2')
    D = batch.n_docs

    def stream(swap=None, dup=None):
        msgs, mrp = [], [0]
        for d in range(D):
            recs = list(range(int(batch.row_ptr[d]), int(batch.row_ptr[d + 1])))
            if d == 1 and swap is not None and len(recs) > swap + 1:
                recs[swap], recs[swap + 1] = recs[swap + 1], recs[swap]
            if d == 1 and dup is not None and len(recs) > dup + 1:
                recs[dup + 1] = recs[dup]
            msgs += [(i, 0, 1, OP, i + 1) for i in recs]
            mrp.append(mrp[-1] + len(recs))
        raw = np.zeros(len(msgs), dtype=RAW_DTYPE)
        for k, f in enumerate(('csn', 'ref_seq', 'client', 'kind', 'op_index')):
            raw[f] = [x[k] for x in msgs]
        return raw, np.array(mrp, dtype=np.uint32)

    assert int(batch.row_ptr[2] - batch.row_ptr[1]) > 20
    raw, mrp = stream()
    TickLog.from_batch(batch, 16, msgs=raw, msg_row_ptr=mrp, pinned=False)  # in order: accepted
    for kw in ({'swap': 3}, {'swap': 15}, {'dup': 7}):  # inside one tick, across ticks 0/1, a repeat
        raw, mrp = stream(**kw)
        with pytest.raises(MtError):
            TickLog.from_batch(batch, 16, msgs=raw, msg_row_ptr=mrp, pinned=False)


def test_layout_on_all_host_cores():
    """Past 4096 documents the layout runs on several host threads (document ranges): the same
    result, checked vectorised -- every record at its tick-major place, every payload byte moved."""
    from fluidframework_amd.oplog import OP_DTYPE, OpBatch
    from fluidframework_amd.ticks import TickLog
    rng = np.random.default_rng(11)
    D, per = 6001, 8
    lens = rng.integers(0, 70, size=D).astype(np.int64)
    n = int(lens.sum())
    ops = np.zeros(n, dtype=OP_DTYPE)
    ops['seq'] = rng.integers(1, 1 << 30, size=n)
    ops['pos1'] = np.arange(n)
    ops['payload_len'] = rng.integers(0, 12, size=n)
    ops['payload_off'] = np.concatenate([[0], np.cumsum(ops['payload_len'].astype(np.int64))[:-1]])
    payload = rng.integers(0, 256, size=int(ops['payload_len'].sum()) + 1).astype(np.uint8)
    row_ptr = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint32)
    batch = OpBatch(ops, payload, row_ptr)
    log = TickLog.from_batch(batch, per, pinned=False)
    doc = np.repeat(np.arange(D), lens)
    j = np.arange(n) - np.repeat(row_ptr[:-1].astype(np.int64), lens)
    t = j // per
    rps = log.row_ptrs.reshape(log.n_ticks, D + 1).astype(np.int64)
    where = log.tick_ops[t].astype(np.int64) + rps[t, doc] + (j - t * per)
    got = log.ops[where]
    assert np.array_equal(got['pos1'], ops['pos1']) and np.array_equal(got['seq'], ops['seq'])
    src = np.repeat(ops['payload_off'].astype(np.int64), ops['payload_len']) + \
        (np.arange(int(ops['payload_len'].sum())) - np.repeat(np.cumsum(ops['payload_len'].astype(np.int64)) -
                                                               ops['payload_len'], ops['payload_len']))
    dst_base = log.tick_payload[t].astype(np.int64) + got['payload_off'].astype(np.int64)
    dst = np.repeat(dst_base, ops['payload_len']) + (src - np.repeat(ops['payload_off'].astype(np.int64),
                                                                      ops['payload_len']))
    assert np.array_equal(log.payload[dst], payload[src])
