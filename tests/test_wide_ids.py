"""Short client ids past a byte and full overlap lists in the wide form (include/mtgpu.h "limits":
MT_MAX_CLIENTS_WIDE, MT_OVX_IDS).  The reference's maps are unbounded
(client.ts:636-660 getOrAddShortClientId, mergeTree.ts:2544-2552 addOverlappingClient); the wide
form holds short ids up to 65534 (254 is NonCollabClient's) and thirty-two overlapping removers >= 64
per segment, and halts a document with MT_DERR_LIMITS past that, as the oracle does.  Reference
pins: tests/golden/wide_many.* (320 clients, 15 overlapping high-id removers on one segment),
wide_xl.* (20 and 32 on one segment;
test_oracle.py / test_gpu_parity.py run every WIDE_SETS entry) and load_wide_many.jsonl (snapshots
with ids past 255, test_snapshot_load.py)."""
import json
import os
import subprocess

import numpy as np
import pytest

from conftest import REPO

MT_DERR_LIMITS = 6


def _overlap_batch(n_high):
    """One document: 300 single-character inserts by clients 1..301 (skipping 254), then n_high
    clients with ids >= 256 remove the same range concurrently: the first takes removedClient, the
    rest overlap it.  A second document stays healthy."""
    from fluidframework_amd.oplog import INSERT, NOOP, OP_DTYPE, REMOVE, OpBatch
    ids = [k for k in range(1, 302) if k != 254]
    recs, payload = [], bytearray()

    def rec(seq, ref, msn, client, typ, p1=0, p2=0, data=b''):
        recs.append((seq, ref, msn, client, typ, 0, p1, p2, len(payload), len(data)))
        payload.extend(data)
    rows = [0]
    for d in range(2):
        s = 0
        for k in ids:
            s += 1
            rec(s, s - 1, 0, k, INSERT, 0, 0, b'abcdefgh'[k % 8:k % 8 + 1])
        base = s
        for j in range(n_high if d == 0 else 3):
            s += 1
            rec(s, base, 0, 256 + j, REMOVE, 10, 20)
        s += 1
        rec(s, s - 1, 0, 1, NOOP)
        rows.append(len(recs))
    return (OpBatch(np.array(recs, dtype=OP_DTYPE), np.frombuffer(bytes(payload), np.uint8),
                    np.array(rows, dtype=np.uint32)), len(ids))


def test_client_interner_skips_noncollab():
    """Hosts intern long client ids to short ids in first-appearance order; 254 is never handed out."""
    from fluidframework_amd.snapshot import ClientInterner
    it = ClientInterner()
    got = [it(f'c{k}') for k in range(300)]
    assert got[:253] == list(range(1, 254)) and got[253] == 255 and 254 not in got
    assert it('c0') == 1  # stable


@pytest.mark.parametrize('n_high', [33, 34])
def test_oracle_overlap_list_limit(oracle_lib, n_high):
    """Thirty-two overlapping removers >= 64 fit (33 removers: one removedClient + 32); the 33rd
    overlap halts the document with MT_DERR_LIMITS at its message, before any of its edits."""
    batch, n_ins = _overlap_batch(n_high)
    o = oracle_lib.Oracle(batch.n_docs).apply(batch)
    if n_high == 33:
        assert o.error(0) == (0, 0)
        ov = max(len([c for c in s[5] if c >= 64]) for s in o.state(0)['segs'])
        assert ov == 32
    else:
        assert o.error(0) == (MT_DERR_LIMITS, n_ins + 34)
    assert o.error(1) == (0, 0)


def test_batchclient_interns_past_254_clients():
    """BatchClient's short ids skip 254 and pass 255 (the wide form's u16 ids); host encoding only."""
    node = '/usr/bin/node' if os.path.exists('/usr/bin/node') else 'node'
    js = ("const {BatchClient}=require('./js/batchClient.js');"
          "const c=new BatchClient({pending:0},0);c.startOrUpdateCollaboration('observer');"
          "for (let i=1;i<=300;i++) c.insertTextRemote(0,'x',undefined,i,i-1,'client'+i);"
          "const q=c.queue.map((r)=>r.client);"
          "console.log(JSON.stringify([q[252],q[253],q[254],q[299],c.getLongClientId(255)]))")
    try:
        out = subprocess.run([node, '-e', js], cwd=REPO, capture_output=True, text=True, timeout=60)
    except OSError:
        pytest.skip('node absent')
    if out.returncode and 'Cannot find module' in out.stderr:
        pytest.skip('node addon absent')
    assert out.returncode == 0, out.stderr
    q = json.loads(out.stdout.strip())
    assert q == [253, 255, 256, 301, 'client254']


@pytest.mark.gpu
@pytest.mark.parametrize('n_high', [33, 34])
def test_engine_overlap_list_limit(oracle_lib, n_high):
    """The device's wide form agrees with the oracle: state at 32 overlapping high-id removers,
    MT_DERR_LIMITS (same message) at 33."""
    from fluidframework_amd.engine import MergeEngine
    batch, _ = _overlap_batch(n_high)
    o = oracle_lib.Oracle(batch.n_docs).apply(batch)
    for b in (0, 32):
        eng = MergeEngine(batch.n_docs, ops_per_launch=b)
        eng.apply(batch)
        for d in range(batch.n_docs):
            assert eng.error(d) == o.error(d), (b, d)
            if o.error(d) == (0, 0):
                assert eng.state(d) == o.state(d), (b, d)
        eng.close()


def _text_on_remove_batch():
    """a remove or annotate record whose payload holds more than its pairs is malformed
    (MT_OP_NO_TEXT_OK): document 0's remove carries two stray bytes, document 1's annotate one."""
    from fluidframework_amd.oplog import ANNOTATE, INSERT, OP_DTYPE, REMOVE, OpBatch
    recs, payload = [], bytearray()

    def rec(seq, ref, client, typ, p1, p2, data, flags=0):
        recs.append((seq, ref, 0, client, typ, flags, p1, p2, len(payload), len(data)))
        payload.extend(data)
    rec(1, 0, 1, INSERT, 0, 0, b'hello')
    rec(2, 1, 2, REMOVE, 1, 3, b'xy')
    rec(1, 0, 1, INSERT, 0, 0, b'hello')
    rec(2, 1, 2, ANNOTATE, 1, 3, b'z' + bytes([1, 5]), 1 << 3)
    return OpBatch(np.array(recs, dtype=OP_DTYPE), np.frombuffer(bytes(payload), np.uint8),
                   np.array([0, 2, 4], dtype=np.uint32))


def test_oracle_rejects_text_on_remove_and_annotate(oracle_lib):
    o = oracle_lib.Oracle(2).apply(_text_on_remove_batch())
    assert o.error(0) == (7, 2) and o.error(1) == (7, 2)


@pytest.mark.gpu
def test_engine_rejects_text_on_remove_and_annotate():
    from fluidframework_amd.engine import MergeEngine
    eng = MergeEngine(2, ops_per_launch=32)
    eng.apply(_text_on_remove_batch())
    assert eng.error(0) == (7, 2) and eng.error(1) == (7, 2)
    eng.close()
