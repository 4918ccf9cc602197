#!/usr/bin/env python3
"""Regenerate the editing-client fixtures FROM THE REFERENCE ITSELF (build container only).

SURVEY.md §8(f) rank 4, local (pending) edits and acks: oracle/tsref/local_farm.js runs reference
Clients c1..c4 editing one document concurrently (insertSegmentLocal / removeRangeLocal /
annotateRangeLocal, client.ts:163-214) behind a toy sequencer and writes the log as c1 sees it --
its own edits as records with seq -1, then the sequenced stream, its own messages coming back as
acks (client.ts:588-625, 804-806; mergeTree.ts:1893-1929; BaseSegment.ack :487-522).
oracle/tsref/replay_ref.js `local` replays each log on a fresh reference Client "c1" and reports
its canonical state at checkpoints (pending segments: seq -1; a pending removal: rseq -1 with its
rclient) and at the end:
  * local_rounds: every client catches up at the end of each round (mergeTreeOperationRunner.ts);
  * local_lag: c1 catches up to a random point only, so its edits interleave with remote ops it
    has not seen yet;
  * local_big: longer lagging runs (zamboni, block splits and packs around pending segments);
  * local_markers: lagging runs whose inserts are Tile / NestBegin / NestEnd markers 15 % of the time;
  * local_reconnect: c1 loses the messages of a round now and then and regenerates them
    (regeneratePendingOp, client.ts:855-893; the client.reconnectFarm.spec.ts pattern): a record
    with seq -2 holds the op being reset, `regen` the ops the reference regenerated from it.
local.expected.jsonl: one JSON line per (log, document): {log, doc, err, states: [[k, state], ...]}
with k the number of the document's records applied.
"""
import json
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
sys.path.insert(0, HERE)

from make_golden import build_log  # noqa: E402

LOGS = (('local_rounds', 24, 11, 300, 0, 6, 0), ('local_lag', 24, 12, 300, 1, 6, 0),
        ('local_big', 16, 13, 1500, 1, 2, 0), ('local_markers', 16, 14, 600, 1, 4, 1),
        ('local_reconnect', 24, 15, 400, 0, 4, 1, 1))
# (name, docs, seed, edits over all clients, lag, checkpoints, markers among the inserts[, reconnects])


def main():
    subprocess.check_call([sys.executable, os.path.join(REPO, 'oracle/tsref/build_ref.py')])
    farm = os.path.join(REPO, 'oracle/tsref/local_farm.js')
    replay = os.path.join(REPO, 'oracle/tsref/replay_ref.js')
    out = []
    for name, n_docs, seed, n_ops, partial, nck, markers, *rc in LOGS:
        reconnect = rc[0] if rc else 0
        res = subprocess.run(['node', farm, str(n_docs), str(seed), str(n_ops), '4', str(partial), str(markers),
                              str(reconnect)], check=True, capture_output=True, text=True)
        docs, farm_regen = [], []
        for recs in json.loads(res.stdout)['docs']:
            if reconnect:
                farm_regen.append(recs['regen'])
                recs = recs['log']
            docs.append([(s, r, m, c, t, p1, p2, text, None if props is None else {int(k): v for k, v in props.items()},
                          flags) for (s, r, m, c, t, p1, p2, text, props, flags) in recs])
        path = os.path.join(HERE, name + '.mtlog')
        build_log(docs).save(path)
        res = subprocess.run(['node', replay, 'local', path, str(nck)], check=True, capture_output=True, text=True)
        for line in res.stdout.strip().split('\n'):
            r = json.loads(line)
            if reconnect:  # the replay regenerated what the farm's client did
                assert r['regen'] == farm_regen[r['doc']], (name, r['doc'])
            out.append(json.dumps(dict(log=name, **r), separators=(',', ':')))
        print(name, len(docs), 'docs', sum(len(d) for d in docs), 'records')
    with open(os.path.join(HERE, 'local.expected.jsonl'), 'w') as f:
        f.write('\n'.join(out) + '\n')
    # the callbacks the reference's editing client fired (local_events.jsonl): in full for the first
    # documents of each log, as count + SHA-256 of the canonical list for the others
    import hashlib
    ev_out = []
    for name, *_ in LOGS:
        res = subprocess.run(['node', replay, 'localevents', os.path.join(HERE, name + '.mtlog')], check=True,
                             capture_output=True, text=True)
        for line in res.stdout.strip().split('\n'):
            r = json.loads(line)
            assert r['err'] is None, (name, r['doc'], r['err'])
            ev = r['events']
            rec = dict(log=name, doc=r['doc'], n=len(ev),
                       sha256=hashlib.sha256(json.dumps(ev, separators=(',', ':')).encode()).hexdigest())
            if r['doc'] < 2:
                rec['events'] = ev
            ev_out.append(json.dumps(rec, separators=(',', ':')))
    with open(os.path.join(HERE, 'local_events.jsonl'), 'w') as f:
        f.write('\n'.join(ev_out) + '\n')
    # SnapshotV1 of editing clients with pending edits (snapshotV1.ts:176-241 elides pending
    # inserts and removals): local_lag cut at its second checkpoint, snapshots by the reference
    from fluidframework_amd.oplog import OpBatch
    import numpy as np
    src = OpBatch.load(os.path.join(HERE, 'local_lag.mtlog'))
    rows = [json.loads(x) for x in out if json.loads(x)['log'] == 'local_lag']
    idx, rp = [], [0]
    for r in rows:
        a, k = int(src.row_ptr[r['doc']]), r['states'][1][0]
        idx.append(np.arange(a, a + k))
        rp.append(rp[-1] + k)
    mid = OpBatch(src.ops[np.concatenate(idx)].copy(), src.payload, np.array(rp, dtype=np.uint32))
    mid.save(os.path.join(HERE, 'local_mid.mtlog'))
    res = subprocess.run(['node', replay, 'snapshot', os.path.join(HERE, 'local_mid.mtlog')], check=True,
                         capture_output=True, text=True)
    with open(os.path.join(HERE, 'local_mid.snapshot.jsonl'), 'w') as f:
        f.write(res.stdout)


if __name__ == '__main__':
    main()
