"""GPU deli ticketing (fluidframework_amd/csrc/mt_deli.hip) through the C-ABI against the CPU
oracle (oracle/deli.py): the lambda.spec.ts known answers, seeded random streams that take every
branch of DeliLambda.ticket, checkpoints (restore / read back), sticky errors, and the fused
deli -> apply hand-off on a synthetic op log.  Bit-exact: every ticket field and every
checkpoint field must match.  Run on the GPU box: python -m pytest tests -m gpu"""
import numpy as np
import pytest

from deli_streams import FIELDS, SPEC, oracle_tickets, random_streams, to_batch
from oracle import deli as od

ERR_CAPACITY = 4  # include/mtgpu.h MT_DELI_ERR_CAPACITY (an engine limit: the oracle has none)

pytestmark = pytest.mark.gpu


def _tickets(t):
    return np.stack([t['seq'], t['msn'], t['ref_seq'], t['status']], axis=1).astype(np.int64)


def _seq(n):
    from fluidframework_amd.deli import DeliSequencer
    return DeliSequencer(n)


def test_lambda_spec_known_answers():
    streams = [s for _, s, _ in SPEC]
    dl = _seq(len(streams))
    got = _tickets(dl.ticket(*to_batch(streams)))
    _, row_ptr = to_batch(streams)
    want, _ = oracle_tickets(streams)
    assert np.array_equal(got, want)
    for d, (name, _, checks) in enumerate(SPEC):
        for i, field, v in checks:
            assert got[row_ptr[d] + i, FIELDS[field]] == v, (name, i, field)


@pytest.mark.parametrize('seed,n_msgs,kw', [(1, 300, {}), (2, 1500, {'n_clients': 40}),
                                            (3, 200, {'n_clients': 64, 'p_assert': 0.02, 'wide': True}),
                                            (4, 64, {}), (5, 65, {'n_clients': 3})])
def test_random_streams_against_oracle(seed, n_msgs, kw):
    streams = random_streams(96, n_msgs, seed=seed, **kw)
    streams[0] = []                                   # an empty document
    want, docs = oracle_tickets(streams)
    dl = _seq(len(streams))
    got = _tickets(dl.ticket(*to_batch(streams)))
    bad = np.nonzero(np.any(got != want, axis=1))[0]
    assert not len(bad), f'{len(bad)} tickets differ, first {int(bad[0])}: got {got[bad[0]]} want {want[bad[0]]}'
    for d in range(len(streams)):
        ck = dl.checkpoint(d)
        o = docs[d].checkpoint()
        assert (ck['seq'], ck['msn'], ck['last_sent_msn'], ck['err']) == (o['seq'], o['msn'], o['last_sent_msn'],
                                                                         o['err']), d
        assert ck['clients'] == o['clients'], d
        if o['err']:
            assert dl.error(d) == (o['err'], docs[d].err_at)


def test_batches_continue_the_state():
    """Two launches over the halves of every stream == one launch over the whole streams."""
    streams = random_streams(64, 700, seed=9, n_clients=20)
    want, _ = oracle_tickets(streams)
    _, rp = to_batch(streams)
    dl = _seq(len(streams))
    a = [s[:len(s) // 2] for s in streams]
    b = [s[len(s) // 2:] for s in streams]
    ta, tb = _tickets(dl.ticket(*to_batch(a))), _tickets(dl.ticket(*to_batch(b)))
    _, rp_a = to_batch(a)
    _, rp_b = to_batch(b)
    for d in range(len(streams)):
        got = np.concatenate([ta[rp_a[d]:rp_a[d + 1]], tb[rp_b[d]:rp_b[d + 1]]])
        assert np.array_equal(got, want[rp[d]:rp[d + 1]]), d


@pytest.mark.parametrize('seed,n_clients,n_msgs', [(11, 96, 1500), (12, 300, 2500), (13, 700, 3000), (14, 2500, 4000)])
def test_documents_past_64_clients_against_oracle(seed, n_clients, n_msgs):
    """Documents whose joined clients pass 63 (96, 300 client ids) or 511 (700, 2500): their first message
    from a client >= 64 promotes them to the wide form (one document per wave, 512 clients), and from a
    client >= 512 on to the huge form (4096), mid-stream; tickets and checkpoints (every client) equal the
    restatement's, in one launch and in two (the promotions and the pools' state carry across calls)."""
    streams = random_streams(48, n_msgs, seed=seed, n_clients=n_clients)
    streams[1] = []
    want, docs = oracle_tickets(streams)
    assert max(c for s in streams for (_, c, _, _) in s) >= (512 if n_clients > 512 else 64)
    # (a deli sized for 16K documents: its huge pool holds 64 of them, more than these streams promote)
    dl = _seq(16384)
    got = _tickets(dl.ticket(*to_batch(streams)))
    bad = np.nonzero(np.any(got != want, axis=1))[0]
    assert not len(bad), f'{len(bad)} tickets differ, first {int(bad[0])}: got {got[bad[0]]} want {want[bad[0]]}'
    for d in range(len(streams)):
        ck, o = dl.checkpoint(d), docs[d].checkpoint()
        assert (ck['seq'], ck['msn'], ck['last_sent_msn'], ck['err']) == (o['seq'], o['msn'], o['last_sent_msn'],
                                                                         o['err']), d
        assert ck['clients'] == o['clients'], d
    # the same streams in two launches
    dl2 = _seq(16384)
    a = [s[:len(s) // 3] for s in streams]
    b = [s[len(s) // 3:] for s in streams]
    ta, tb = _tickets(dl2.ticket(*to_batch(a))), _tickets(dl2.ticket(*to_batch(b)))
    _, rp = to_batch(streams)
    _, rp_a = to_batch(a)
    _, rp_b = to_batch(b)
    for d in range(len(streams)):
        two = np.concatenate([ta[rp_a[d]:rp_a[d + 1]], tb[rp_b[d]:rp_b[d + 1]]])
        assert np.array_equal(two, want[rp[d]:rp[d + 1]]), d
        assert dl2.checkpoint(d)['clients'] == docs[d].checkpoint()['clients'], d


def test_big_pool_exhausted_halts_the_document():
    """The big pool holds max(64, max_docs / 16) documents past client 63: with 80 such documents the
    80 - 64 promoted last halt at the message that needed a row (MT_DELI_ERR_CAPACITY -- an engine
    limit, told apart from a bad client id -- the rest of their tickets HALTED); the others are
    ticketed as the restatement does."""
    streams = []
    for d in range(80):
        s = [(od.JOIN, c, -1, -1) for c in range(60, 70)] + [(od.OP, 65, 1, 10), (od.OP, 61, 1, 11)]
        streams.append(s)
    want, _ = oracle_tickets(streams)
    dl = _seq(len(streams))
    got = _tickets(dl.ticket(*to_batch(streams)))
    _, rp = to_batch(streams)
    halted = [d for d in range(80) if dl.error(d)[0]]
    assert len(halted) == 16, halted
    for d in range(80):
        g, w = got[rp[d]:rp[d + 1]], want[rp[d]:rp[d + 1]]
        if d in halted:
            assert dl.error(d) == (ERR_CAPACITY, 4)  # the join of client 64
            assert np.array_equal(g[:4], w[:4]) and np.all(g[4:, 3] == od.HALTED), d
        else:
            assert np.array_equal(g, w), d


def test_huge_pool_exhausted_halts_the_document():
    """The huge pool holds max(8, max_docs / 256) documents past client 511: of 12 documents that join
    client 600, the 4 promoted last halt at that join (MT_DELI_ERR_CAPACITY); the rest, promoted through
    the big pool to the huge one, are ticketed as the restatement does."""
    streams = [[(od.JOIN, c, -1, -1) for c in (5, 70, 600)] + [(od.OP, 600, 1, 3), (od.OP, 70, 1, 4)]
               for _ in range(12)]
    want, docs = oracle_tickets(streams)
    dl = _seq(len(streams))
    got = _tickets(dl.ticket(*to_batch(streams)))
    _, rp = to_batch(streams)
    halted = [d for d in range(12) if dl.error(d)[0]]
    assert len(halted) == 4, halted
    for d in range(12):
        g, w = got[rp[d]:rp[d + 1]], want[rp[d]:rp[d + 1]]
        if d in halted:
            assert dl.error(d) == (ERR_CAPACITY, 2)  # the join of client 600
            assert np.array_equal(g[:2], w[:2]) and np.all(g[2:, 3] == od.HALTED), d
        else:
            assert np.array_equal(g, w), d
            assert dl.checkpoint(d)['clients'] == docs[d].checkpoint()['clients'], d


def test_big_pool_rows_come_back_on_restore():
    """Restoring a promoted document gives its big-pool row back (a free list the next promotion takes
    first): 64 documents fill the pool, 16 of them are restored, and 16 new documents then promote
    without MT_DELI_ERR_CAPACITY; a row is never shared (every document's tickets as the restatement's)."""
    def wide_stream(d):
        return [(od.JOIN, c, -1, -1) for c in range(60, 70)] + [(od.OP, 65, 1, 10 + d % 3), (od.OP, 61, 1, 11)]
    n = 128  # max(64, n / 16) = 64 rows
    first = [wide_stream(d) if d < 64 else [] for d in range(n)]
    dl = _seq(n)
    dl.ticket(*to_batch(first))
    _, first_docs = oracle_tickets(first)
    assert all(dl.error(d)[0] == 0 for d in range(64))
    dl.restore([{'seq': 0, 'clients': {}, 'last_sent_msn': 0}] * 16, doc0=8)  # documents 8..23 back to new
    assert all(dl.checkpoint(d)['clients'] == {} for d in range(8, 24))
    second = [wide_stream(d) if 64 <= d < 80 else [] for d in range(n)]
    want, docs = oracle_tickets(second)
    got = _tickets(dl.ticket(*to_batch(second)))
    assert np.array_equal(got, want)
    assert all(dl.error(d)[0] == 0 for d in range(n))
    for d in list(range(64, 80)) + [0, 7, 24, 63]:  # the new rows, and rows the restore left alone
        assert dl.checkpoint(d)['clients'] == (docs[d] if d >= 64 else first_docs[d]).checkpoint()['clients'], d
    # one more promotion finds the pool full again
    third = [wide_stream(d) if d == 100 else [] for d in range(n)]
    dl.ticket(*to_batch(third))
    assert dl.error(100) == (ERR_CAPACITY, 4)


@pytest.mark.parametrize('seed,n_clients', [(31, 96), (32, 300), (33, 700)])
def test_wide_checkpoint_round_trip(seed, n_clients):
    """generateDeliCheckpoint / restore of documents past client 63: the narrow checkpoint call refuses
    them (MT_ERR_WIDE, nothing dropped), the wide one carries every client, and a deli restored from it
    tickets the rest of the stream as the restatement does (the msn derived over all clients)."""
    from fluidframework_amd.engine import MtError
    streams = random_streams(24, 1200, seed=seed, n_clients=n_clients)
    half = [s[:len(s) // 2] for s in streams]
    rest = [s[len(s) // 2:] for s in streams]
    dl = _seq(8192)
    dl.ticket(*to_batch(half))
    _, docs = oracle_tickets(half)
    cks = []
    for d in range(len(streams)):
        ck, o = dl.checkpoint(d), docs[d].checkpoint()
        assert ck['clients'] == o['clients'] and (ck['seq'], ck['msn']) == (o['seq'], o['msn']), d
        if max(o['clients'], default=0) >= 64:
            with pytest.raises(MtError, match='wide'):
                dl.checkpoint_narrow(d)
        else:
            assert dl.checkpoint_narrow(d)['clients'] == o['clients'], d
        cks.append({'seq': ck['seq'], 'clients': ck['clients'], 'last_sent_msn': ck['last_sent_msn']})
    assert any(max(c['clients'], default=0) >= 64 for c in cks)
    want, _ = oracle_tickets(rest, checkpoints=cks)
    dl2 = _seq(8192)
    dl2.restore(cks)
    for d in range(len(streams)):
        got_ck = dl2.checkpoint(d)
        assert got_ck['clients'] == cks[d]['clients'] and got_ck['msn'] == od.DeliDoc(**cks[d]).msn, d
    assert np.array_equal(_tickets(dl2.ticket(*to_batch(rest))), want)


def test_restore_from_checkpoints():
    streams = random_streams(32, 400, seed=21, n_clients=30)
    cks = []
    for d, s in enumerate(streams):
        doc = od.DeliDoc()
        for m in s[:len(s) // 2]:
            doc.ticket(*m)
        ck = doc.checkpoint()
        cks.append({'seq': ck['seq'], 'clients': ck['clients'], 'last_sent_msn': ck['last_sent_msn']})
    rest = [s[len(s) // 2:] for s in streams]
    want, _ = oracle_tickets(rest, checkpoints=cks)
    dl = _seq(len(streams))
    dl.restore(cks)
    assert np.array_equal(_tickets(dl.ticket(*to_batch(rest))), want)


def test_deli_feeds_apply():
    """C5's hand-off: raw op messages from a synthetic op log (every client joined at seq 0),
    deli re-derives each op's seq / msn from (client, csn, refSeq) alone and stamps them into the
    staged op records, and the apply engine replays the stamped log into the generator's state
    (the synthetic msn is deli's: min over the clients' latest refSeq)."""
    from fluidframework_amd.deli import RAW_DTYPE, TICKET_DTYPE, batch_device_ptrs
    from fluidframework_amd.engine import MergeEngine
    from fluidframework_amd.hipmem import DeviceBuffer
    from fluidframework_amd.oplog import CONFIGS
    cfg = dict(CONFIGS['C3'])
    cfg.pop('n_docs')
    cfg['ops_per_doc'] = 256
    n = 512
    eng = MergeEngine(n, ops_per_launch=32)
    dev = eng.synthesize(seed=3, **cfg)
    want_cs = eng.checksums()
    host = dev.to_host()
    d_ops, _, d_row = batch_device_ptrs(dev)
    msgs = DeviceBuffer(dev.n_ops * RAW_DTYPE.itemsize)
    tick = DeviceBuffer(dev.n_ops * TICKET_DTYPE.itemsize)
    dl = _seq(n)
    dl.restore_all(seq=0, clients={c: (0, 0, False) for c in range(1, cfg['n_clients'] + 1)})
    dl.raw_from_ops(d_ops, d_row, n, msgs.ptr)
    dl.ticket_device(msgs.ptr, d_row, n, tick.ptr, d_ops, dev.n_ops)
    dl.sync()
    raw = msgs.download(RAW_DTYPE)
    assert np.array_equal(raw['ref_seq'], host.ops['ref_seq']) and np.all(raw['kind'] == od.OP)
    t = tick.download(TICKET_DTYPE)
    assert np.all(t['status'] == od.SENT)
    assert np.array_equal(t['seq'], host.ops['seq']) and np.array_equal(t['msn'], host.ops['msn'])
    assert np.array_equal(dev.to_host().ops, host.ops)
    eng.reset()
    eng.apply_staged(dev)
    assert np.array_equal(eng.checksums(), want_cs)


def test_c5_joins_through_deli_then_apply(oracle_lib):
    """BASELINE config C5 as specified: per document, the ClientJoin of its 8
    clients and then its 256 op messages -- raw messages, no pre-seeded checkpoint -- ticketed on
    the GPU from new documents (lambda.ts:286-299: each join revs the sequence number), seq / msn /
    refSeq stamped into the op records (fused hand-off), then applied.  Checked against the deli
    restatement (oracle/deli.py, ticket by ticket) feeding the merge-tree oracle (oracle/mtcpu.cpp,
    checksum by checksum) on 1,024 documents."""
    from fluidframework_amd.deli import RAW_DTYPE, TICKET_DTYPE, batch_device_ptrs
    from fluidframework_amd.engine import MergeEngine
    from fluidframework_amd.hipmem import DeviceBuffer
    from fluidframework_amd.oplog import CONFIGS
    cfg = dict(CONFIGS['C5'])
    cfg.pop('n_docs')
    n, n_join = 1024, cfg['n_clients']
    eng = MergeEngine(n, ops_per_launch=32)
    dev = eng.synthesize(seed=5, **cfg)
    host = dev.to_host()
    d_ops, _, d_row = batch_device_ptrs(dev)
    n_msgs = dev.n_ops + n * n_join
    msgs = DeviceBuffer(n_msgs * RAW_DTYPE.itemsize)
    mrow = DeviceBuffer((n + 1) * 4)
    tick = DeviceBuffer(n_msgs * TICKET_DTYPE.itemsize)
    dl = _seq(n)
    dl.restore_all(seq=0, clients={})
    dl.raw_stream(d_ops, d_row, n, n_join, msgs.ptr, mrow.ptr)
    dl.ticket_device(msgs.ptr, mrow.ptr, n, tick.ptr, d_ops, dev.n_ops)
    dl.sync()
    raw = msgs.download(RAW_DTYPE)
    rp = mrow.download(np.uint32)
    assert rp[0] == 0 and rp[-1] == n_msgs
    for d in (0, 1, n - 1):   # joins of clients 1..8 first, then the log's ops with refSeq + 8
        seg = raw[rp[d]:rp[d + 1]]
        assert list(seg['kind'][:n_join]) == [od.JOIN] * n_join and list(seg['client'][:n_join]) == list(range(1, 9))
        ops = host.ops[host.row_ptr[d]:host.row_ptr[d + 1]]
        assert np.array_equal(seg['ref_seq'][n_join:], ops['ref_seq'] + n_join)
        assert np.array_equal(seg['op_index'][n_join:], np.arange(host.row_ptr[d], host.row_ptr[d + 1]) + 1)
    want, _ = od.ticket_batch(raw, rp)
    got = _tickets(tick.download(TICKET_DTYPE))
    bad = np.nonzero(np.any(got != want, axis=1))[0]
    assert not len(bad), f'{len(bad)} tickets differ, first {int(bad[0])}: {got[bad[0]]} vs {want[bad[0]]}'
    assert np.all(want[:, 3] == od.SENT)
    # the oracle's stamped log: each op record gets its message's ticket
    stamped = host.ops.copy()
    link = raw['op_index'] > 0
    k = raw['op_index'][link].astype(np.int64) - 1
    stamped['seq'][k], stamped['msn'][k], stamped['ref_seq'][k] = want[link, 0], want[link, 1], want[link, 2]
    assert np.array_equal(dev.to_host().ops, stamped)
    assert np.array_equal(stamped['seq'], host.ops['seq'] + n_join)
    from fluidframework_amd.oplog import OpBatch
    o = oracle_lib.Oracle(n).apply(OpBatch(stamped, host.payload, host.row_ptr), threads=8)
    eng.reset()
    eng.apply_staged(dev)
    assert np.array_equal(eng.checksums(), o.checksums())
    assert all(eng.error(d) == (0, 0) for d in range(0, n, 97))


def test_c5_tick_feed_through_deli(oracle_lib):
    """C5's raw streams as a tick-major feed from page-locked host memory (mt_submit_ticks_deli):
    tick 0 carries every document's 8 joins and first 32 op messages, each later tick the next 32;
    each tick is ticketed by deli on the engine's stream (fused stamping into the tick's records)
    and then applied, with the next ticks' copies in flight.  Tickets and final states equal the
    HBM-resident deli -> apply of the whole stream (itself pinned to the oracles above)."""
    from fluidframework_amd.deli import RAW_DTYPE, TICKET_DTYPE, batch_device_ptrs
    from fluidframework_amd.engine import MergeEngine
    from fluidframework_amd.hipmem import DeviceBuffer
    from fluidframework_amd.oplog import CONFIGS
    from fluidframework_amd.ticks import TickLog
    cfg = dict(CONFIGS['C5'])
    cfg.pop('n_docs')
    n, n_join = 1536, cfg['n_clients']
    eng = MergeEngine(n, ops_per_launch=32)
    dev = eng.synthesize(seed=7, **cfg)
    host = dev.to_host()
    d_ops, _, d_row = batch_device_ptrs(dev)
    n_msgs = dev.n_ops + n * n_join
    msgs = DeviceBuffer(n_msgs * RAW_DTYPE.itemsize)
    mrow = DeviceBuffer((n + 1) * 4)
    tick = DeviceBuffer(n_msgs * TICKET_DTYPE.itemsize)
    dl = _seq(n)
    dl.restore_all(seq=0, clients={})
    dl.raw_stream(d_ops, d_row, n, n_join, msgs.ptr, mrow.ptr)
    dl.sync()
    raw, rp = msgs.download(RAW_DTYPE), mrow.download(np.uint32)
    dl.ticket_device(msgs.ptr, mrow.ptr, n, tick.ptr, d_ops, dev.n_ops)
    dl.sync()
    want_t = tick.download(TICKET_DTYPE)
    eng.reset()
    eng.apply_staged(dev)
    want_cs = eng.checksums()
    for b, first in ((32, None), (16, None), (32, 8)):
        log = TickLog.from_batch(host, 32, msgs=raw, msg_row_ptr=rp, tickets=True, first=first)
        assert log.n_ticks == (8 if first is None else 10)  # (ramp 8, 16, then 32s)
        e2 = MergeEngine(n, ops_per_launch=b)
        dl.restore_all(seq=0, clients={})
        e2.apply_ticks(log, deli=dl)
        assert np.array_equal(e2.checksums(), want_cs), b
        # the tickets, back in each document's order
        got = np.zeros(n_msgs, dtype=TICKET_DTYPE)
        for d in range(n):
            parts = []
            for t in range(log.n_ticks):
                r = log.msg_row_ptrs[t * (n + 1):(t + 1) * (n + 1)]
                m0 = int(log.tick_msgs[t])
                parts.append(log.tickets[m0 + int(r[d]):m0 + int(r[d + 1])])
            got[rp[d]:rp[d + 1]] = np.concatenate(parts)
        assert np.array_equal(_tickets(got), _tickets(want_t))
        assert all(e2.error(d) == (0, 0) for d in range(0, n, 97))
        e2.close()
        log.free()


def test_unsent_messages_halt_the_document(oracle_lib):
    """a message deli does not send (here a csn gap and a refSeq below the msn, both
    nacked, lambda.ts:269-275, 319-335) stamps MT_SEQ_NACK into its op record, never the local-edit
    seq -1: the apply engine halts that document with MT_DERR_SEQ_ORDER at that record instead of
    applying the nacked op as a pending local edit; the other documents replay unchanged."""
    from fluidframework_amd.deli import RAW_DTYPE, TICKET_DTYPE, batch_device_ptrs
    from fluidframework_amd.engine import MergeEngine
    from fluidframework_amd.hipmem import DeviceBuffer
    from fluidframework_amd.oplog import CONFIGS, OpBatch
    cfg = dict(CONFIGS['C3'])
    cfg.pop('n_docs')
    cfg['ops_per_doc'] = 256
    n = 64
    eng = MergeEngine(n, ops_per_launch=32)
    dev = eng.synthesize(seed=11, **cfg)
    host = dev.to_host()
    d_ops, _, d_row = batch_device_ptrs(dev)
    msgs = DeviceBuffer(dev.n_ops * RAW_DTYPE.itemsize)
    tick = DeviceBuffer(dev.n_ops * TICKET_DTYPE.itemsize)
    dl = _seq(n)
    dl.restore_all(seq=0, clients={c: (0, 0, False) for c in range(1, cfg['n_clients'] + 1)})
    dl.raw_from_ops(d_ops, d_row, n, msgs.ptr)
    dl.sync()
    raw = msgs.download(RAW_DTYPE)
    rp = host.row_ptr.astype(np.int64)
    raw['csn'][rp[0] + 100] += 5                      # doc 0: a gap in the sender's csn
    j = rp[1] + 150                                   # doc 1: a refSeq below the msn
    assert host.ops['msn'][j - 1] > 0
    raw['ref_seq'][j] = int(host.ops['msn'][j - 1]) - 1
    msgs.upload(raw)
    dl2 = _seq(n)
    dl2.restore_all(seq=0, clients={c: (0, 0, False) for c in range(1, cfg['n_clients'] + 1)})
    dl2.ticket_device(msgs.ptr, d_row, n, tick.ptr, d_ops, dev.n_ops)
    dl2.sync()
    docs = [od.DeliDoc(seq=0, clients={c: (0, 0, False) for c in range(1, cfg['n_clients'] + 1)}) for _ in range(n)]
    want, _ = od.ticket_batch(raw, host.row_ptr, docs)
    got = _tickets(tick.download(TICKET_DTYPE))
    assert np.array_equal(got, want)
    assert want[rp[0] + 100, 3] != od.SENT and want[j, 3] != od.SENT
    stamped = host.ops.copy()
    sent = want[:, 3] == od.SENT
    stamped['seq'] = np.where(sent, want[:, 0], -3)   # MT_SEQ_NACK
    stamped['msn'], stamped['ref_seq'] = want[:, 1], want[:, 2]
    assert np.array_equal(dev.to_host().ops, stamped)
    eng.reset()
    eng.apply_staged(dev)
    o = oracle_lib.Oracle(n).apply(OpBatch(stamped, host.payload, host.row_ptr), threads=8)
    assert eng.error(0) == (1, -3) and eng.error(1) == (1, -3)
    assert all(eng.error(d) == o.error(d) for d in range(n))
    assert np.array_equal(eng.checksums(), o.checksums())
