"""HIP engine (libmtgpu.so) parity on an MI355X: bit-exact against the reference's golden
outputs (tests/golden, produced by the reference itself) and against the CPU oracle on fresh
synthetic logs.  Run on the GPU box:  python -m pytest tests -m gpu"""
import numpy as np
import pytest

from conftest import FULLSHAPE_SETS, GOLDEN_SETS, WIDE_SETS, load_fullshape, load_golden

pytestmark = pytest.mark.gpu


def _diff(a, b):
    if a == b:
        return None
    for k in ('seq', 'msn', 'tree'):
        if a[k] != b[k]:
            return f'{k}: {a[k]} != {b[k]}'
    for i, (x, y) in enumerate(zip(a['segs'], b['segs'])):
        if x != y:
            return f'seg {i}: {x} != {y}'
    return f'nsegs {len(a["segs"])} != {len(b["segs"])}'


@pytest.mark.parametrize('b', [0, 32, 5])
@pytest.mark.parametrize('name', GOLDEN_SETS + WIDE_SETS)
def test_golden_bit_exact(name, b):
    from fluidframework_amd.engine import MergeEngine
    batch, exp = load_golden(name)
    eng = MergeEngine(batch.n_docs, ops_per_launch=b)
    eng.apply(batch)
    cs = eng.checksums()
    for r in exp:
        d = r['doc']
        assert eng.error(d) == (0, 0), (name, d, eng.error(d))
        st = eng.state(d)
        assert st == r['state'], f'{name} doc {d} b={b}: {_diff(st, r["state"])}'
        assert eng.text(d) == r['text']
        assert '%016x' % cs[d] == r['checksum']


@pytest.mark.parametrize('name', WIDE_SETS + ['scenarios'])
def test_tick_feed_golden(name):
    """The golden sets through the tick feed (mt_submit_ticks, 16 ops per document per tick): the
    wide sets' first ticks hold wide records, which the device-side check of the first tick must
    report (the wide form's workspace is set up from it) -- the reference's states."""
    from fluidframework_amd.engine import MergeEngine
    from fluidframework_amd.ticks import TickLog
    batch, exp = load_golden(name)
    log = TickLog.from_batch(batch, 16)
    eng = MergeEngine(batch.n_docs, ops_per_launch=16)
    eng.apply_ticks(log)
    cs = eng.checksums()
    for r in exp:
        d = r['doc']
        assert eng.error(d) == (0, 0), (name, d, eng.error(d))
        assert '%016x' % cs[d] == r['checksum'], (name, d)
    eng.close()
    log.free()


@pytest.mark.parametrize('b', [0, 32, 5])
@pytest.mark.parametrize('name', FULLSHAPE_SETS)
def test_fullshape_bit_exact(name, b):
    """The engine against the reference itself at the benchmark configs' full shape (C3, C4: 256
    documents x 1024 ops; C5: 1,024 documents x 256 ops; C3 with 48 clients, the C64 form) and on a fixed-seed 1,000-document x 1024-op high-conflict fuzz
    (tests/golden/make_fullshape.py): every document's checksum of the reference's canonical state,
    and the first documents' states whole, at launch sizes 0 (one launch), 32 and 5."""
    from fluidframework_amd.engine import MergeEngine
    batch, fx = load_fullshape(name)
    eng = MergeEngine(batch.n_docs, ops_per_launch=b)
    eng.apply(batch)
    got = ['%016x' % c for c in eng.checksums()]
    bad = [d for d in range(batch.n_docs) if got[d] != fx['checksum'][d]]
    assert not bad, f'{name} b={b}: {len(bad)} documents differ, first {bad[:5]}: {eng.error(bad[0])}'
    for d, st in fx['states'].items():
        assert eng.state(int(d)) == st, f'{name} doc {d} b={b}: {_diff(eng.state(int(d)), st)}'
    assert all(eng.error(d) == (0, 0) for d in range(0, batch.n_docs, 7))


@pytest.mark.parametrize('per,b,first', [(32, 32, None), (64, 32, None), (5, 0, None), (32, 32, 8), (32, 32, 1)])
@pytest.mark.parametrize('name', ['full_c4', 'fuzz_1k'])
def test_tick_feed_equals_reference(name, per, b, first):
    """mt_submit_ticks (the tick-major feed: later ticks copied from page-locked host memory into a
    ring of device slots while tick k applies) ends in the reference's states, as mt_submit does:
    ticks of 32 ops per document applied as one launch, ticks of 64 as two launches of 32, ticks of
    5 in one launch each (hundreds of ticks: the ring wraps many times), and a short first tick
    (mt_log_to_ticks_ramp)."""
    from fluidframework_amd.engine import MergeEngine
    from fluidframework_amd.ticks import TickLog
    batch, fx = load_fullshape(name)
    log = TickLog.from_batch(batch, per, first=first)
    eng = MergeEngine(batch.n_docs, ops_per_launch=b)
    eng.apply_ticks(log)
    got = ['%016x' % c for c in eng.checksums()]
    bad = [d for d in range(batch.n_docs) if got[d] != fx['checksum'][d]]
    assert not bad, f'{name} per={per}: {len(bad)} documents differ, first {bad[:5]}: {eng.error(bad[0])}'
    # launches and algorithmic bytes cover the whole call
    _, _, launches, nbytes = eng.last_stats()
    assert launches >= log.n_ticks and nbytes > 0
    # the same feed again after a reset: the ring is reused
    eng.reset()
    eng.apply_ticks(log)
    assert ['%016x' % c for c in eng.checksums()] == got
    eng.close()
    log.free()


def test_tick_feed_stops_at_a_malformed_tick():
    """A tick whose payload bounds are broken is refused (MT_ERR_ARG) with the ticks before it applied,
    as a loop of applyMsg stops at the message that throws."""
    from fluidframework_amd.engine import MergeEngine, MtError
    from fluidframework_amd.ticks import TickLog
    batch, fx = load_golden('synth_c2')
    log = TickLog.from_batch(batch, 16)
    t2 = log.tick_batch(2)
    t2.ops['payload_off'][0] = 1 << 30
    t2.ops['payload_len'][0] = 4
    ref = MergeEngine(batch.n_docs, ops_per_launch=16)
    for t in range(2):
        ref.apply(log.tick_batch(t))
    eng = MergeEngine(batch.n_docs, ops_per_launch=16)
    with pytest.raises(MtError):
        eng.apply_ticks(log)
    assert np.array_equal(eng.checksums(), ref.checksums())


@pytest.mark.parametrize('where', ['first', 'last'])
def test_tick_feed_refuses_a_malformed_first_tick(where):
    """The first tick's records are checked on the device once they have landed
    (mt_scan_records_kernel, not on the host before the copy): a payload out of bounds there -- at
    its first or its last record -- refuses the feed with nothing applied; the same feed repaired then
    applies as before (wide records in the first tick: tests/test_wide_ids.py)."""
    from fluidframework_amd.engine import MergeEngine, MtError
    from fluidframework_amd.ticks import TickLog
    batch, fx = load_golden('synth_c2')
    log = TickLog.from_batch(batch, 16)
    t0 = log.tick_batch(0)
    i = 0 if where == 'first' else len(t0.ops) - 1
    keep = t0.ops[i].copy()
    t0.ops['payload_off'][i] = int(log.tick_payload[1] - log.tick_payload[0])  # one past the tick's payload
    t0.ops['payload_len'][i] = 1
    eng = MergeEngine(batch.n_docs, ops_per_launch=16)
    empty = eng.checksums()
    with pytest.raises(MtError):
        eng.apply_ticks(log)
    assert np.array_equal(eng.checksums(), empty)
    t0.ops[i] = keep
    eng.reset()
    eng.apply_ticks(log)
    ref = MergeEngine(batch.n_docs, ops_per_launch=16)
    ref.apply(batch)
    assert np.array_equal(eng.checksums(), ref.checksums())


@pytest.mark.parametrize('cfg_name', ['C2', 'C3', 'C4'])
def test_fuzz_against_oracle(oracle_lib, cfg_name):
    from fluidframework_amd.engine import MergeEngine
    from fluidframework_amd.oplog import CONFIGS
    cfg = dict(CONFIGS[cfg_name])
    cfg.pop('n_docs')
    n = 256
    batch = oracle_lib.generate(n, seed=1234, **cfg)
    o = oracle_lib.Oracle(n).apply(batch, threads=8)
    eng = MergeEngine(n, ops_per_launch=32)
    eng.apply(batch)
    want, got = o.checksums(), eng.checksums()
    bad = np.nonzero(want != got)[0]
    if len(bad):
        d = int(bad[0])
        pytest.fail(f'{len(bad)}/{n} docs differ; doc {d}: err={eng.error(d)} {_diff(eng.state(d), o.state(d))}')
    assert all(eng.error(d) == (0, 0) for d in range(0, n, 17))


@pytest.mark.parametrize('cfg_name', ['C2', 'C3', 'C4'])
def test_device_generator_matches_host_generator(oracle_lib, cfg_name):
    """The bench's on-device op synthesis (mt_synth.h, GEN kernel) emits exactly the log the
    oracle's host generator emits; replaying it from empty reproduces the generation state."""
    from fluidframework_amd.engine import MergeEngine
    from fluidframework_amd.oplog import CONFIGS
    cfg = dict(CONFIGS[cfg_name])
    cfg.pop('n_docs')
    cfg['ops_per_doc'] = 512
    n = 96
    eng = MergeEngine(n)
    dev = eng.synthesize(seed=99, **cfg)
    gen_cs = eng.checksums()
    host = oracle_lib.generate(n, seed=99, **cfg)
    got = dev.to_host()
    for f in ('seq', 'ref_seq', 'msn', 'client', 'type', 'flags', 'pos1', 'pos2', 'payload_len'):
        assert np.array_equal(got.ops[f], host.ops[f]), f
    for d in range(n):
        a = got.doc_slice(d, d + 1)
        b = host.doc_slice(d, d + 1)
        assert np.array_equal(a.payload, b.payload), d
    eng.reset()
    eng.apply_staged(dev)
    assert np.array_equal(eng.checksums(), gen_cs)
    o = oracle_lib.Oracle(n).apply(host, threads=8)
    assert np.array_equal(o.checksums(), gen_cs)


@pytest.mark.parametrize('name,chunk', [('scenarios', None), ('synth_c1', None), ('synth_c3', None),
                                        ('synth_c4', None), ('synth_tiny', None), ('synth_c3', 300)])
def test_snapshot_matches_reference(name, chunk):
    """mt_get_snapshot (device extraction + host JSON) == the tree the reference's SnapshotV1
    emitted for the same log (tests/golden/*.snapshot*.jsonl)."""
    from fluidframework_amd.engine import MergeEngine
    from test_snapshot import load_snapshots
    batch, _ = load_golden(name)
    eng = MergeEngine(batch.n_docs, ops_per_launch=32)
    eng.apply(batch)
    names = ['observer'] + ['c%d' % i for i in range(1, 64)]
    want = load_snapshots(name, chunk)
    for d, w in enumerate(want):
        assert eng.snapshot(d, chunk or 0, names) == w['snapshot'], (name, d)
    # the batched, multithreaded form (mt_get_snapshots) of every document at once
    assert eng.snapshots(0, batch.n_docs, chunk or 0, names) == [w['snapshot'] for w in want], name


def test_snapshot_matches_restatement_on_fuzz(oracle_lib):
    """Random config-shaped logs (no reference run): engine snapshot == oracle/snapshot.py on the
    oracle's state, at the default and a small chunk size."""
    from fluidframework_amd.engine import MergeEngine
    from oracle import snapshot
    batch = oracle_lib.generate(48, seed=99, n_clients=12, ops_per_doc=700, max_lag=48, n_keys=3, n_values=4,
                                p_insert=0.55, p_remove=0.3, p_overlap=0.4, p_null=0.2, p_insert_props=0.3)
    o = oracle_lib.Oracle(48).apply(batch, threads=8)
    eng = MergeEngine(48, ops_per_launch=32)
    eng.apply(batch)
    names = ['observer'] + ['c%d' % i for i in range(1, 64)]
    for d in range(48):
        st = o.state(d)
        for chunk in (0, 97):
            assert eng.snapshot(d, chunk, names) == snapshot.emit(st, chunk or snapshot.DEFAULT_CHUNK), d
    for chunk in (0, 97):
        got = eng.snapshots(5, 40, chunk, names)
        for i, d in enumerate(range(5, 45)):
            assert got[i] == snapshot.emit(o.state(d), chunk or snapshot.DEFAULT_CHUNK), (chunk, d)


@pytest.mark.parametrize('b', [32, 7])
def test_wide_and_narrow_documents_share_an_engine(oracle_lib, b):
    """Wide documents (tests/golden/wide*: UTF-16 text, 120 client ids, u16 value ids, keys 8..15) in
    one engine with narrow C3 documents on the register engine: each kind on its own form, both
    bit-exact; the narrow documents' checksums equal the oracle's."""
    from fluidframework_amd.engine import MergeEngine
    from fluidframework_amd.oplog import CONFIGS, OpBatch
    cfg = dict(CONFIGS['C3'])
    cfg.pop('n_docs')
    cfg['ops_per_doc'] = 400
    narrow = oracle_lib.generate(64, seed=8, **cfg)
    wides = [load_golden(n) for n in WIDE_SETS]
    batch = OpBatch.concat([narrow] + [w for w, _ in wides])
    eng = MergeEngine(batch.n_docs, ops_per_launch=b)
    eng.apply(batch)
    o = oracle_lib.Oracle(64).apply(narrow, threads=8)
    assert np.array_equal(eng.checksums()[:64], o.checksums())
    d0 = 64
    for w, exp in wides:
        for r in exp:
            d = d0 + r['doc']
            assert eng.error(d) == (0, 0), (d, eng.error(d))
            assert eng.state(d) == r['state'], _diff(eng.state(d), r['state'])
            assert eng.text(d) == r['text']
        d0 += w.n_docs


def test_narrow_documents_promote_to_wide_mid_batch(oracle_lib):
    """Narrow C3 documents replayed halfway, then a wide record (a CJK insert, a client id >= 64, a
    value id past 255, or a key past 7) arrives: each document moves to the wide form with its state
    (text widened in place of the arena) and the rest of its log applies bit-exact with the oracle."""
    from fluidframework_amd.engine import MergeEngine
    from fluidframework_amd.oplog import CONFIGS, OP_WIDE, OpBatch, INSERT, ANNOTATE
    cfg = dict(CONFIGS['C3'])
    cfg.pop('n_docs')
    cfg['ops_per_doc'] = 512
    n = 48
    full = oracle_lib.generate(n, seed=19, **cfg)
    # the same logs with one record per document turned wide at op 256
    ops = full.ops.copy()
    payload = bytearray(full.payload.tobytes())
    for d in range(n):
        i = int(full.row_ptr[d]) + 256
        o = ops[i]
        kind = d % 4
        if kind == 1 and o['type'] != 3:
            ops[i]['client'] = 64 + d          # a client id >= 64 (its first appearance)
            continue
        # rewrite the record as a wide insert of two CJK units (payload appended)
        text = '中文'.encode('utf-16-le')
        pairs = b''
        if kind == 2:
            pairs = bytes([1, 0x2C, 0x01])     # key 1 -> value id 300
        elif kind == 3:
            pairs = bytes([11, 5, 0])          # key 11 -> value id 5
        off = len(payload)
        payload += text + pairs
        ops[i]['type'] = INSERT | OP_WIDE
        ops[i]['flags'] = (2 | (1 << 3)) if pairs else 0
        ops[i]['pos1'] = 0
        ops[i]['payload_off'] = off
        ops[i]['payload_len'] = len(text) + len(pairs)
    batch = OpBatch(ops, np.frombuffer(bytes(payload), np.uint8), full.row_ptr)
    o = oracle_lib.Oracle(n).apply(batch, threads=8)
    eng = MergeEngine(n, ops_per_launch=32)
    eng.apply(batch)
    got, want = eng.checksums(), o.checksums()
    bad = np.nonzero(got != want)[0]
    assert len(bad) == 0, [(int(d), eng.error(int(d)), o.error(int(d)), _diff(eng.state(int(d)), o.state(int(d))))
                           for d in bad[:3]]
    assert all(eng.error(d) == o.error(d) for d in range(n))
