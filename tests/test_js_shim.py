"""The Node host surface (js/batchClient.js over the N-API addon js/mtgpu.node)."""
import json
import os
import shutil
import subprocess

import pytest

from conftest import GOLDEN, REPO, load_golden

NODE = shutil.which('node')
pytestmark = pytest.mark.skipif(not NODE, reason='node not installed')


def _addon():
    from fluidframework_amd import build
    build.build()
    return build.build_napi()


def test_addon_loads_and_exports():
    if not _addon():
        pytest.skip('node headers absent')
    out = subprocess.run([NODE, '-e', "const b=require('./js/batchClient.js');"
                          "for (const f of ['createEngine','submit','submitAsync','getText','getState','getLength',"
                          "'docError','checksums','version','eventsEnable','eventsDrain','findTiles','rangeStacks','docsLoad','regenDrain','setLabelKeys']) if (typeof b.native[f] !== 'function') throw f;"
                          "console.log(b.native.version())"], cwd=REPO, capture_output=True, text=True)
    assert out.returncode == 0, out.stderr
    assert 'gfx950' in out.stdout


def _to_log_ids(state):
    def cid(x):
        return 0 if x == 'observer' else int(x[1:])
    segs = []
    for text, seq, c, rseq, rc, ov, props in state['segs']:
        segs.append([text, seq, cid(c), rseq, cid(rc) if rc != -1 else -1, sorted(cid(o) for o in ov),
                     None if props is None else {k: v for k, v in sorted(props.items(), key=lambda kv: int(kv[0][1:]))}])
    return dict(state, segs=segs)


@pytest.mark.gpu
@pytest.mark.parametrize('name', ['scenarios', 'synth_c3', 'synth_tiny', 'wide', 'wide_synth'])
def test_batchclient_replays_golden(name):
    assert _addon()
    _, exp = load_golden(name)
    out = subprocess.run([NODE, os.path.join(REPO, 'js', 'replay_golden.js'), os.path.join(GOLDEN, name + '.mtlog'),
                          '32'], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-2000:]
    got = [json.loads(x) for x in out.stdout.strip().split('\n')]
    for r, e in zip(got, exp):
        assert r['text'] == e['text']
        # getLength: UTF-16 code units of the live segments, a marker counting 1 (getText skips markers)
        assert r['length'] == sum(1 if isinstance(sg[0], dict) else len(sg[0].encode('utf-16-le', 'surrogatepass')) // 2
                                  for sg in e['state']['segs'] if sg[3] == -1)
        assert _to_log_ids(r['state']) == e['state'], (name, r['doc'])


def test_addon_exports_deli():
    if not _addon():
        pytest.skip('node headers absent')
    out = subprocess.run([NODE, '-e', "const n=require('./js/mtgpu.node');"
                          "for (const f of ['createDeli','deliTicket','deliError']) if (typeof n[f] !== 'function') throw f;"
                          "require('./js/deliSequencer.js');"], cwd=REPO, capture_output=True, text=True)
    assert out.returncode == 0, out.stderr


@pytest.mark.gpu
def test_deli_sequencer_replays_lambda_spec():
    """lambda.spec.ts's scenarios as IRawOperationMessages through js/deliSequencer.js: the
    asserted MSN values (0, 1, 4, 7, 7 and 20, 22) and nacks."""
    assert _addon()
    out = subprocess.run([NODE, os.path.join(REPO, 'js', 'deli_spec.js')], capture_output=True, text=True,
                         timeout=120)
    assert out.returncode == 0, out.stderr[-2000:]
    docs = [json.loads(x) for x in out.stdout.strip().split('\n')]
    disconnect, above, nacked = docs
    assert [disconnect[i][2] for i in (0, 3, 5, 6, 8)] == [0, 1, 4, 7, 7]
    assert all(r[0] == 'sent' for r in disconnect)
    assert above[2][2] == 20 and above[5][2] == 22
    assert nacked[3][0] == 'nack' and nacked[3][3].startswith('Refseq')
    assert nacked[4][0] == 'nack' and nacked[4][3] == 'Nonexistent client'


def test_batchclient_encodes_wide_records():
    """Text is UTF-16 code units (textSegment.ts:45 cachedLength = text.length): Latin-1 text goes out
    narrow (one byte per unit); CJK or a surrogate pair -- or a value id past 255, a key past 7 -- makes
    the record wide (MT_OP_WIDE: 2 bytes per unit, 3-byte pairs).  No device work: host encoding only."""
    if not _addon():
        pytest.skip('node headers absent')
    js = ("const {BatchClient}=require('./js/batchClient.js');"
          "const c=new BatchClient({pending:0},0);c.startOrUpdateCollaboration('observer');"
          "c.insertTextRemote(0,'caf\\u00e9',undefined,1,0,'w');"
          "c.insertTextRemote(0,'\\u4e2d\\u6587',undefined,2,1,'w');"
          "c.insertTextRemote(0,'a\\ud83d\\ude00b',{k:1},3,2,'w');"
          "const props={};for (let i=0;i<300;i++) props['v'+i]=undefined;"
          "for (let i=0;i<300;i++) c.applyMsg(c.makeOpMessage({type:2,pos1:0,pos2:1,props:{m:'id'+i}},4+i,3,'w'));"
          "const q=c.queue.map((r)=>[r.type,r.flags,r.payload.length]);"
          "console.log(JSON.stringify([q[0],q[1],q[2],q[3+254],q[3+255]]))")
    out = subprocess.run([NODE, '-e', js], cwd=REPO, capture_output=True, text=True)
    assert out.returncode == 0, out.stderr
    q = json.loads(out.stdout.strip())
    assert q[0] == [0, 0, 4]                       # narrow: 4 Latin-1 bytes
    assert q[1] == [0x80, 0, 4]                    # wide: 2 units x 2 bytes
    assert q[2] == [0x80, 2, 8 + 3]                # wide: a, surrogate pair, b = 4 units; one 3-byte pair
    assert q[3] == [2, 0, 2]                       # value id 255 of key "m": a narrow pair
    assert q[4] == [0x82, 0, 3]                    # value id 256: a wide annotate


@pytest.mark.gpu
def test_flush_async_in_order_then_sync_read():
    """submitAsync runs on a libuv pool thread; two unawaited flushAsync() and a sync
    getText() must not overlap on the engine: batches apply once each, in flush order."""
    assert _addon()
    out = subprocess.run([NODE, os.path.join(REPO, 'js', 'async_order.js')], capture_output=True, text=True,
                         timeout=120)
    assert out.returncode == 0, out.stderr[-2000:]
    r = json.loads(out.stdout)
    # every insert at position 0 with refSeq = seq - 1 lands in front: the text is the inserts
    # of the document in reverse seq order
    seq, want = 0, [[] for _ in range(4)]
    for _ in range(6):
        for d in range(4):
            for _ in range(5):
                seq += 1
                want[d].append(chr(97 + seq % 26))
    assert r['text'] == [''.join(reversed(w)) for w in want]
    assert r['length'] == [30] * 4


@pytest.mark.gpu
def test_deli_reuses_short_ids_after_leave():
    """200 sessions (join, 2 ops, leave) of one document through DeliSequencer: ids of
    processed leaves are reused, every op is sent, the leave of a never-seen client is dropped."""
    assert _addon()
    out = subprocess.run([NODE, os.path.join(REPO, 'js', 'deli_reuse.js')], capture_output=True, text=True,
                         timeout=120)
    assert out.returncode == 0, out.stderr[-2000:]
    r = json.loads(out.stdout)
    assert r['statuses'] == {'dropped': 1, 'sent': 800}
    assert r['seq'] == 800 and r['interned'] == 0


@pytest.mark.gpu
@pytest.mark.parametrize('name', ['scenarios', 'markers', 'errors', 'empty_inserts', 'synth_tiny', 'synth_c4', 'wide',
                                  'wide_synth'])
def test_batchclient_delivers_reference_callbacks(name):
    """mergeTreeDeltaCallback / mergeTreeMaintenanceCallback on BatchClient (flushes every 40
    messages, 32 ops per launch) deliver exactly the callbacks the reference's own Client fired
    (tests/golden/events.jsonl, make_events.py), in order, with propertyDeltas un-interned."""
    from test_events import _err_seqs, _golden_events, _matches
    assert _addon()
    gold = _golden_events()[name]
    errs = _err_seqs(name)
    _, exp = load_golden(name)
    out = subprocess.run([NODE, os.path.join(REPO, 'js', 'replay_golden.js'), os.path.join(GOLDEN, name + '.mtlog'),
                          '32', 'events'], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-2000:]
    got = [json.loads(x) for x in out.stdout.strip().split('\n')]
    for r in got:
        d = r['doc']
        assert _matches(gold[d], r['events'], errs.get(d)), (name, d)
        assert (r['err'] is None) == (errs.get(d) is None), (name, d)
        assert _to_log_ids(r['state']) == exp[d]['state'], (name, d)


def _js_state_to_log(state):
    """BatchClient.getState (long client ids "c<k>", "observer"; -2 = NonCollabClient) in the golden
    logs' id space; property names and values as they are."""
    def cid(x):
        return x if isinstance(x, int) else (0 if x == 'observer' else int(x[1:]))
    segs = [[t, sq, cid(c), rs, cid(rc) if rc != -1 else -1, sorted(cid(o) for o in ov), p]
            for t, sq, c, rs, rc, ov, p in state['segs']]
    return dict(state, segs=segs)


@pytest.mark.gpu
@pytest.mark.parametrize('name', ['scenarios', 'synth_c3', 'synth_c4', 'markers', 'synth_markers'])
def test_batchclient_loads_reference_snapshots(name):
    """js/snapshotLoader.js (SnapshotLoader over mt_docs_load + MT_OP_LOAD appends): the snapshot
    the reference emitted after messages [0, k), loaded into BatchClients, then messages [k, n):
    the reference's state after the same (tests/golden/load_<set>.jsonl)."""
    from test_snapshot_load import err_code, load_set
    assert _addon()
    rows = load_set(name)
    out = subprocess.run([NODE, os.path.join(REPO, 'js', 'replay_load.js'), 'sets',
                          os.path.join(GOLDEN, f'load_{name}.jsonl'), os.path.join(GOLDEN, name + '.mtlog'), '32'],
                         capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-2000:]
    got = {r['doc']: r for r in (json.loads(x) for x in out.stdout.strip().split('\n'))}
    for r in rows:
        g = got[r['doc']]
        assert (g['err'] is None) == (err_code(r['err']) == 0), (name, r['doc'], g['err'], r['err'])
        if r['state'] is not None:
            assert _js_state_to_log(g['state']) == r['state'], (name, r['doc'])


@pytest.mark.gpu
def test_batchclient_loads_reference_snapshot_files():
    """All 15 of the reference's own snapshot test files (v1 / legacy / legacy with catch-up ops;
    header-only, header + body, large body, annotated, markers with a markerId each) through
    BatchClient: the loaded state, then the spec's edits."""
    from test_snapshot_load import REF_DIR, err_code
    assert _addon()
    with open(os.path.join(REF_DIR, 'expected.jsonl')) as f:
        cases = {c['file']: c for c in (json.loads(x) for x in f if x.strip())}
    out = subprocess.run([NODE, os.path.join(REPO, 'js', 'replay_load.js'), 'files',
                          os.path.join(REF_DIR, 'expected.jsonl'), REF_DIR], capture_output=True, text=True,
                         timeout=300)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [json.loads(x) for x in out.stdout.strip().split('\n')]
    assert len(lines) == 15
    for g in lines:
        c = cases[g['file']]
        assert _js_state_to_log(g['loaded']) == c['loaded'], g['file']
        assert (g['err'] is None) == (err_code(c['err']) == 0), g['file']
        assert _js_state_to_log(g['state']) == c['state'], g['file']


@pytest.mark.gpu
@pytest.mark.parametrize('name', ['tiles_scenarios', 'tiles_synth', 'tiles_annot'])
def test_batchclient_find_tile_matches_reference(name):
    """BatchClient.findTile (mt_find_tiles via the addon; label arrays interned by content) gives
    the reference Client.findTile answers of tests/golden/tiles.expected.jsonl."""
    from test_tiles import load_tiles
    assert _addon()
    out = subprocess.run([NODE, os.path.join(REPO, 'js', 'replay_tiles.js'), os.path.join(GOLDEN, name + '.mtlog'),
                          os.path.join(GOLDEN, 'tiles.expected.jsonl'), name, '0'], capture_output=True, text=True,
                         timeout=300)
    assert out.returncode == 0, out.stderr[-2000:]
    got = {r['doc']: r['answers'] for r in (json.loads(x) for x in out.stdout.strip().split('\n'))}
    for r in load_tiles()[name]:
        assert got[r['doc']] == r['answers'], (name, r['doc'])


@pytest.mark.gpu
@pytest.mark.parametrize('name', ['tiles_scenarios', 'tiles_synth', 'tiles_annot'])
def test_batchclient_stack_context_matches_reference(name):
    """BatchClient.getStackContext (mt_range_stacks via the addon) gives the reference
    Client.getStackContext stacks of tests/golden/stacks.expected.jsonl."""
    from test_stacks import load_stacks
    assert _addon()
    out = subprocess.run([NODE, os.path.join(REPO, 'js', 'replay_stacks.js'), os.path.join(GOLDEN, name + '.mtlog'),
                          os.path.join(GOLDEN, 'stacks.expected.jsonl'), name, '1'], capture_output=True, text=True,
                         timeout=300)
    assert out.returncode == 0, out.stderr[-2000:]
    got = {r['doc']: r['answers'] for r in (json.loads(x) for x in out.stdout.strip().split('\n'))}
    for r in load_stacks()[name]:
        assert got[r['doc']] == r['answers'], (name, r['doc'])


@pytest.mark.gpu
@pytest.mark.parametrize('name', ['local_rounds', 'local_lag', 'local_big', 'local_markers', 'local_reconnect'])
def test_batchclient_editing_client_matches_reference(name):
    """BatchClient as an editing client (insertTextLocal / removeRangeLocal / annotateRangeLocal,
    its own sequenced messages as acks through applyMsg, regeneratePendingOp on reconnect) ends
    every local_* document in the reference client's final state and regenerates the reference's
    ops (tests/golden/local.expected.jsonl)."""
    from test_local import load_local
    assert _addon()
    out = subprocess.run([NODE, os.path.join(REPO, 'js', 'replay_local.js'), os.path.join(GOLDEN, name + '.mtlog')],
                         capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-2000:]
    got = {r['doc']: r for r in (json.loads(x) for x in out.stdout.strip().split('\n'))}
    for r in load_local()[name]:
        g = got[r['doc']]
        assert g['err'] is None, (name, r['doc'], g['err'])
        assert _js_state_to_log(g['state']) == r['states'][-1][1], (name, r['doc'])
        assert g.get('regen', []) == r.get('regen', []), (name, r['doc'])  # regeneratePendingOp


@pytest.mark.gpu
@pytest.mark.parametrize('name', ['local_lag', 'local_reconnect'])
def test_batchclient_editing_client_callbacks_match_reference(name):
    """mergeTreeDeltaCallback / mergeTreeMaintenanceCallback on an editing BatchClient: its local
    edits' callbacks (no sequencedMessage), remote ops' and zamboni's, in order -- the reference's
    (tests/golden/local_events.jsonl)."""
    import hashlib
    assert _addon()
    out = subprocess.run([NODE, os.path.join(REPO, 'js', 'replay_local.js'), os.path.join(GOLDEN, name + '.mtlog'),
                          'events'], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-2000:]
    got = {r['doc']: r for r in (json.loads(x) for x in out.stdout.strip().split('\n'))}
    with open(os.path.join(GOLDEN, 'local_events.jsonl')) as f:
        gold = [json.loads(x) for x in f if json.loads(x)['log'] == name]
    for g in gold:
        ev = got[g['doc']]['events']
        if 'events' in g:
            assert ev == g['events'], (name, g['doc'])
        assert len(ev) == g['n'] and hashlib.sha256(json.dumps(ev, separators=(',', ':')).encode()).hexdigest() == \
            g['sha256'], (name, g['doc'])


SEQDELTA_LOGS = ['seqdelta', 'local_rounds', 'local_lag', 'local_big', 'local_markers', 'local_reconnect', 'scenarios',
                 'markers', 'wide', 'synth_c1']


def _seqdelta_gold():
    with open(os.path.join(GOLDEN, 'seqdelta.expected.jsonl')) as f:
        return [json.loads(x) for x in f if x.strip()]


def test_seqdelta_fixture_covers_the_spec():
    """tests/golden/seqdelta.expected.jsonl holds the reference's SequenceDeltaEvents for every `it` of
    sequenceDeltaEvent.spec.ts (59 documents) and for the editing / observer logs; spot-check facts the
    spec asserts (positions after a concurrent remote edit, two ranges for a split removal)."""
    gold = _seqdelta_gold()
    assert {g['log'] for g in gold} == set(SEQDELTA_LOGS)
    spec = [g for g in gold if g['log'] == 'seqdelta']
    assert len(spec) == 59 and all(g['err'] is None for g in spec)
    # collab insert "separate regions, local before remote": the remote insert lands at 23 + 12
    ev = spec[3]['events']
    assert ev[1][2] is True and ev[1][5] == [[0, 1, 4, 12, None]]
    assert ev[2][2] is False and ev[2][5][0][2] == 35 and ev[2][5][0][3] == 5
    # combination "insertPos is deleteRangeStart, insertLocal deleteRemote": "brown " and "fox " as two ranges
    two = [e for g in spec for e in g['events'] if e[1] == 1 and len(e[5]) == 2 and e[5][0][3] == 6 and e[5][1][3] == 4]
    assert two and two[0][5][1][2] == 4 + 11
    # .ranges "multiple noncontinuous segments": the remote remove's five ranges at 4, 8, ..., 20
    last = spec[-1]['events'][-1]
    assert last[2] is False and [r[2] for r in last[5]] == [4, 8, 12, 16, 20]


def test_sequence_events_install_and_remove_callbacks():
    """SequenceEvents (js/sequenceDeltaEvent.js) installs the client's callback with the first listener,
    wraps each callback in a SequenceDeltaEvent (ranges sorted by ordinal, one per segment, isLocal
    without a sequenced message) and uninstalls with the last listener -- no device needed."""
    src = r"""
const { SequenceEvents, SequenceDeltaEvent } = require('./js/sequenceDeltaEvent.js');
const client = { longClientId: 'c7' };
const seq = new SequenceEvents(client);
if (client.mergeTreeDeltaCallback) throw 'installed early';
const seen = [];
const fn = (ev) => seen.push(ev);
seq.on('sequenceDelta', fn);
const s = (ordinal, position, cachedLength) => ({ ordinal, position, cachedLength });
client.mergeTreeDeltaCallback({ sequencedMessage: undefined }, { operation: 2, deltaSegments: [
    { segment: s(5, 9, 2), propertyDeltas: { k0: null } }, { segment: s(3, 4, 1), propertyDeltas: { k0: 1 } },
    { segment: s(5, 9, 2), propertyDeltas: { k0: 7 } }] });
client.mergeTreeDeltaCallback({ sequencedMessage: { sequenceNumber: 4 } }, { operation: 1, deltaSegments: [] });
const [a, b] = seen;
if (!(a instanceof SequenceDeltaEvent) || !a.isLocal || a.isEmpty || a.clientId !== 'c7') throw 'event a';
if (a.ranges.map((r) => r.segment.ordinal).join() !== '3,5' || a.first.position !== 4 || a.last.position !== 9) throw 'ranges';
if (a.ranges[1].propertyDeltas.k0 !== null || a.ranges[0].operation !== 2) throw 'first range per segment';
if (b.isLocal || !b.isEmpty || b.first !== undefined || b.deltaOperation !== 1) throw 'event b';
seq.off('sequenceDelta', fn);
if (client.mergeTreeDeltaCallback) throw 'not uninstalled';
console.log('ok');
"""
    out = subprocess.run([NODE, '-e', src], cwd=REPO, capture_output=True, text=True)
    assert out.returncode == 0 and out.stdout.strip() == 'ok', out.stderr


@pytest.mark.gpu
@pytest.mark.parametrize('name', SEQDELTA_LOGS)
def test_batchclient_sequence_delta_events_match_reference(name):
    """SequenceDeltaEvents ("sequenceDelta" listeners of js/sequenceDeltaEvent.js over an editing or
    observer BatchClient): operation, isLocal, isEmpty, clientId, every range's leaf / position /
    cachedLength / propertyDeltas and first / last, read in the listener -- the reference's
    SequenceDeltaEvent over the reference client (tests/golden/seqdelta.expected.jsonl; seqdelta.mtlog is
    sequenceDeltaEvent.spec.ts re-expressed as logs)."""
    import hashlib
    assert _addon()
    out = subprocess.run([NODE, os.path.join(REPO, 'js', 'replay_local.js'), os.path.join(GOLDEN, name + '.mtlog'),
                          'seqdelta'], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-2000:]
    got = {r['doc']: r for r in (json.loads(x) for x in out.stdout.strip().split('\n'))}
    gold = [g for g in _seqdelta_gold() if g['log'] == name]
    assert gold
    for g in gold:
        ev = got[g['doc']]['events']
        if 'events' in g:
            assert ev == g['events'], (name, g['doc'])
        else:
            assert len(ev) == g['n'] and hashlib.sha256(json.dumps(ev, separators=(',', ':')).encode()).hexdigest() == \
                g['sha256'], (name, g['doc'])


SEQREADS_LOGS = {'seqdelta': None, 'local_lag': 6, 'local_rounds': 6, 'local_markers': 4, 'scenarios': 12}


def _seqreads_gold():
    with open(os.path.join(GOLDEN, 'seqreads.expected.jsonl')) as f:
        return [json.loads(x) for x in f if x.strip()]


def test_seqreads_fixture_covers_the_spec():
    """seqreads.expected.jsonl (tests/golden/make_seqreads.py, the transpiled reference): every document of
    seqdelta.mtlog (sequenceDeltaEvent.spec.ts re-expressed) in full, with local and remote callbacks, and
    reads that change between callbacks."""
    gold = _seqreads_gold()
    assert {g['log'] for g in gold} == set(SEQREADS_LOGS)
    spec = [g for g in gold if g['log'] == 'seqdelta']
    assert len(spec) == 59 and all(g['err'] is None and g['n'] == len(g['reads']) for g in spec)
    seqs = {r[0] for g in spec for r in g['reads']}
    assert -1 in seqs and any(x > 0 for x in seqs)
    assert any(len({r[1] for r in g['reads']}) > 2 for g in spec)
    assert any(len(r[3]) > 1 for g in spec for r in g['reads'])


@pytest.mark.gpu
@pytest.mark.parametrize('name', sorted(SEQREADS_LOGS))
def test_batchclient_sync_callbacks_read_reference_state(name):
    """BatchEngine({syncCallbacks: true}): a listener reading getText() / getLength() / getPosition(segment)
    of its delta segments INSIDE the callback reads what the reference's listener reads inside the
    reference's callback (tests/golden/seqreads.expected.jsonl)."""
    import hashlib
    assert _addon()
    n = SEQREADS_LOGS[name]
    out = subprocess.run([NODE, os.path.join(REPO, 'js', 'replay_local.js'), os.path.join(GOLDEN, name + '.mtlog'),
                          'seqreads'] + ([str(n)] if n else []), capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-2000:]
    got = {r['doc']: r for r in (json.loads(x) for x in out.stdout.strip().split('\n'))}
    gold = [g for g in _seqreads_gold() if g['log'] == name]
    assert gold
    for g in gold:
        reads = got[g['doc']]['reads']
        if 'reads' in g:
            assert reads == g['reads'], (name, g['doc'])
        else:
            assert len(reads) == g['n'] and hashlib.sha256(json.dumps(reads, separators=(',', ':')).encode()).hexdigest() \
                == g['sha256'], (name, g['doc'])


READ_LOGS = ['scenarios', 'markers', 'synth_markers', 'wide', 'synth_c1', 'local_lag', 'local_markers',
             'local_reconnect']


def _read_gold():
    with open(os.path.join(GOLDEN, 'read.expected.jsonl')) as f:
        return [json.loads(x) for x in f if x.strip()]


def test_read_fixture_covers_logs():
    gold = _read_gold()
    assert {g['log'] for g in gold} == set(READ_LOGS)
    full = [g for g in gold if 'contain' in g]
    assert full and all(g['err'] is None for g in full)
    # the fixture exercises misses (positions past the end), props, stopped walks and unresolvable
    # remote positions
    assert any(x is None for g in full for x in g['contain'])
    assert any(x is not None for g in full for x in g['props'])
    assert any(len(g['walks'][2]) == 3 for g in full)
    assert any(r[3] is None for g in full for r in g['remote'])


@pytest.mark.gpu
@pytest.mark.parametrize('name', READ_LOGS)
def test_batchclient_read_surface_matches_reference(name):
    """getContainingSegment / getPropertiesAtPosition / getRangeExtentsOfPosition, walkSegments,
    getPosition and resolveRemoteClientPosition on BatchClient over the device state equal the
    reference client's on the same logs (tests/golden/read.expected.jsonl, make_read.py)."""
    import hashlib
    assert _addon()
    out = subprocess.run([NODE, os.path.join(REPO, 'js', 'replay_local.js'), os.path.join(GOLDEN, name + '.mtlog'),
                          'read'], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-2000:]
    got = {r['doc']: r for r in (json.loads(x) for x in out.stdout.strip().split('\n'))}
    gold = [g for g in _read_gold() if g['log'] == name]
    assert gold
    for g in gold:
        r = got[g['doc']]
        if 'sha256' in g:
            assert hashlib.sha256(json.dumps(r, separators=(',', ':')).encode()).hexdigest() == g['sha256'], \
                (name, g['doc'])
        else:
            e = {k: v for k, v in g.items() if k != 'log'}
            for k in e:
                assert r[k] == e[k], (name, g['doc'], k)


@pytest.mark.gpu
def test_batchclient_get_marker_from_id_on_reference_snapshots():
    """getMarkerFromId (client.ts:311-313) after loading the reference's withMarkers snapshots (564
    markers, each with its markerId): every id resolves to its marker at its position in the
    reference loader's state; an unknown id to undefined."""
    from test_snapshot_load import REF_DIR
    assert _addon()
    with open(os.path.join(REF_DIR, 'expected.jsonl')) as f:
        cases = {c['file']: c for c in (json.loads(x) for x in f if x.strip())}
    out = subprocess.run([NODE, os.path.join(REPO, 'js', 'replay_load.js'), 'markers',
                          os.path.join(REF_DIR, 'expected.jsonl'), REF_DIR], capture_output=True, text=True,
                         timeout=300)
    assert out.returncode == 0, out.stderr[-2000:]
    n_markers = 0
    for g in (json.loads(x) for x in out.stdout.strip().split('\n')):
        segs = cases[g['file']]['loaded']['segs']
        exp, pos = [], 0
        for i, s in enumerate(segs):
            live = s[4] == -1
            if isinstance(s[0], dict) and s[6] and 'markerId' in s[6]:
                exp.append([s[6]['markerId'], i, pos, s[0]['marker']])
            if live:
                pos += 1 if isinstance(s[0], dict) else len(s[0].encode('utf-16-le', 'surrogatepass')) // 2
        exp.append(['no such marker', None])
        assert g['found'] == exp, g['file']
        n_markers += len(exp) - 1
    assert n_markers >= 3 * 564
