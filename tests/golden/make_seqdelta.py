#!/usr/bin/env python3
"""SequenceDeltaEvent fixtures FROM THE REFERENCE ITSELF (build container only; needs /root/reference and node).

SURVEY.md §8(f) row f3: packages/dds/sequence/src/test/sequenceDeltaEvent.spec.ts re-expressed as op
logs -- every `it` of its "non-collab", "collab" (insert / delete / annotate / combination) and
"SequenceDeltaEvent .ranges" suites is one document whose editing client is "c1" (the spec's
localUser) and whose remote user is "c2".  The spec's starting text (inserted before collaboration)
is a sequenced insert by c2 at seq 1; after it, each step is the spec's: a local edit (record seq -1),
its ack (the spec's makeOpMessage of the local op) and the remote ops, at the spec's seq / refSeq.
Property names map to key ids (foo 0, foo1 1, foo2 2, foo3 3) and values to value ids (bar 1, bar1 2,
bar2 3, bar3 4, bardash 5).
oracle/tsref/replay_ref.js `seqdelta` replays each log on a reference Client and builds the reference's
SequenceDeltaEvent (sequence/src/sequenceDeltaEvent.ts, transpiled) in every delta callback; the
record of an event is [seq (-1: local edit), deltaOperation, isLocal, isEmpty, clientId, ranges
[[operation, leaf, position, cachedLength, propertyDeltas | null], ...], first leaf, last leaf].
seqdelta.expected.jsonl: {log, doc, err, n, events} in full for seqdelta.mtlog and for the first
documents of the local_* / observer logs, {log, doc, err, n, sha256} (of the canonical event list)
for the others.  Fixtures are data only (inputs and reference outputs).
"""
import hashlib
import json
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
sys.path.insert(0, HERE)

from make_golden import A, I, R, build_log  # noqa: E402

ME, THEM = 1, 2
FOO, FOO1, FOO2, FOO3 = 0, 1, 2, 3
BAR, BAR1, BAR2, BAR3, BARDASH = 1, 2, 3, 4, 5


def op(kind, *a):
    """a spec edit: ('i', pos, text) / ('r', start, end) / ('a', start, end, props)"""
    return (kind,) + a


def rec(o, seq, ref, client):
    if o[0] == 'i':
        return I(seq, ref, 0, client, o[1], o[2])
    if o[0] == 'r':
        return R(seq, ref, 0, client, o[1], o[2])
    return A(seq, ref, 0, client, o[1], o[2], o[3])


class Doc:
    """one spec `it`: records in the order the spec applies them"""

    def __init__(self, text=None):
        self.recs = []
        self.cur = 0
        if text:
            self.recs.append(I(1, 0, 0, THEM, 0, text))
            self.cur = 1

    def local(self, o):
        self.recs.append(rec(o, -1, self.cur, ME))

    def msg(self, o, seq, ref, client):
        self.recs.append(rec(o, seq, ref, client))
        self.cur = max(self.cur, seq)

    def pair(self, local, remote, local_first):
        """the collab pattern: a local edit and a remote edit, both at refSeq cur; "local before
        remote" acks the local one at cur+1 and sequences the remote one at cur+2, "remote before
        local" the other way round"""
        c = self.cur
        self.local(local)
        if local_first:
            self.msg(local, c + 1, c, ME)
            self.msg(remote, c + 2, c, THEM)
        else:
            self.msg(remote, c + 1, c, THEM)
            self.msg(local, c + 2, c, ME)
        return self


def spec_docs():
    docs = []
    # non-collab (:29-210): local edits on a client that never hears back
    d = Doc()
    for pos, text in ((0, 'done'), (0, "What's "), (11, ' done'), (11, ' is')):
        d.local(op('i', pos, text))
    docs.append(d)
    d = Doc('All is well!')
    for a, b in ((3, 7), (0, 3), (4, 5), (0, 4)):
        d.local(op('r', a, b))
    docs.append(d)
    d = Doc('All is well!')
    for a, b, p in ((0, 3, {FOO1: BAR1}), (3, 7, {FOO2: BAR2}), (7, 12, {FOO3: BAR3}), (2, 10, {FOO: BAR}),
                    (2, 10, {FOO: None}), (2, 3, {FOO1: None}), (3, 7, {FOO2: None}), (7, 10, {FOO3: None})):
        d.local(op('a', a, b, p))
    docs.append(d)
    # collab insert (:217-672), base "The fox jumps over the dog"
    fox = 'The fox jumps over the dog'
    for lo, ro in ((op('i', 4, 'quick brown '), op('i', 23, 'lazy ')), (op('i', 23, 'lazy '), op('i', 4, 'quick brown ')),
                   (op('i', 4, 'brown '), op('i', 4, 'quick ')), (op('i', 4, 'quick '), op('i', 4, 'brown ')),
                   (op('i', 4, 'quick brown '), op('i', 3, ' legendary')),
                   (op('i', 3, ' legendary'), op('i', 4, 'quick brown '))):
        for first in (True, False):
            docs.append(Doc(fox).pair(lo, ro, first))
    d = Doc(fox)  # multiple inserts: local, remote, remoteAfterLocal (:527-598)
    d.local(op('i', 4, 'brown '))
    d.msg(op('i', 4, 'brown '), 2, 1, ME)
    d.msg(op('i', 4, 'quick '), 3, 1, THEM)
    d.msg(op('i', 35, 'lazy '), 4, 2, THEM)
    docs.append(d)
    d = Doc(fox)  # multiple inserts: remote, local, localAfterRemote (:600-671)
    d.local(op('i', 4, 'quick '))
    d.msg(op('i', 4, 'brown '), 2, 1, THEM)
    d.msg(op('i', 4, 'quick '), 3, 1, ME)
    d.local(op('i', 35, 'lazy '))
    d.msg(op('i', 35, 'lazy '), 4, 2, ME)
    docs.append(d)
    # collab delete (:674-1280), base "The quick brown fox jumps over the lazy dog"
    qb = 'The quick brown fox jumps over the lazy dog'
    for (la, lb), (ra, rb) in (((4, 10), (35, 40)), ((4, 16), (4, 16)), ((4, 16), (10, 15)), ((4, 10), (9, 16)),
                               ((9, 16), (4, 10)), ((10, 15), (4, 16))):
        for first in (True, False):
            docs.append(Doc(qb).pair(op('r', la, lb), op('r', ra, rb), first))
    # collab annotate (:1282-1945), base "Habits change into character"
    hab = 'Habits change into character'
    for lp, rp in (({FOO: BAR}, {FOO: BAR}), ({FOO: BAR}, {FOO: BARDASH}), ({FOO1: BAR1}, {FOO2: BAR2})):
        for first in (True, False):
            docs.append(Doc(hab).pair(op('a', 7, 13, lp), op('a', 7, 13, rp), first))
    d = Doc(hab)  # overlapping ranges, same properties, different values (:1611-1945)
    d.local(op('a', 7, 13, {FOO1: BAR1}))
    d.msg(op('a', 7, 13, {FOO1: BAR1}), 2, 1, ME)
    d.local(op('a', 19, 28, {FOO3: BAR3}))
    d.msg(op('a', 19, 28, {FOO3: BAR3}), 3, 2, ME)
    d.msg(op('a', 14, 18, {FOO2: BAR2}), 4, 1, THEM)
    d.msg(op('a', 0, 28, {FOO: BAR}), 5, 4, THEM)                 # step1
    d.local(op('a', 0, 13, {FOO: BAR1}))                          # step2
    d.msg(op('a', 0, 13, {FOO: BAR1}), 6, 5, ME)
    d.msg(op('a', 14, 28, {FOO: BAR2}), 7, 5, THEM)               # step3 (has not seen step2)
    d.local(op('a', 7, 28, {FOO: BAR3}))                          # step4
    d.msg(op('a', 7, 28, {FOO: BAR3}), 8, 7, ME)
    docs.append(d)
    # combination (:1947-2995), base "The brown fox jumps over the lazy dog"
    bf = 'The brown fox jumps over the lazy dog'
    for ip, it, da, db in ((4, 'quick ', 29, 34), (29, 'black ', 4, 10), (29, 'black ', 29, 34), (34, 'black ', 29, 34),
                           (10, 'black wolf ', 4, 14)):
        for ins_local in (True, False):
            for first in (True, False):
                ins, rem = op('i', ip, it), op('r', da, db)
                docs.append(Doc(bf).pair(ins, rem, first) if ins_local else Doc(bf).pair(rem, ins, first))
    # SequenceDeltaEvent .ranges (:2998-3093)
    d = Doc()
    d.local(op('i', 0, 'text'))
    docs.append(d)
    d = Doc()
    for _ in range(7):
        d.local(op('i', 0, 'text'))
    d.local(op('a', 4, 24, {FOO: BAR}))
    docs.append(d)
    d = Doc()
    for i in range(5):
        d.local(op('i', 0, str(i) * 4))
        d.msg(op('i', 0, str(i) * 4), i + 1, i, ME)
    for i in range(5):
        d.local(op('i', i * 8, 'bbbb'))
    d.msg(op('r', 0, 20), 6, 5, THEM)
    docs.append(d)
    return build_log([x.recs for x in docs])


FULL_DOCS = 3  # documents of the other logs stored in full
LOGS = ('local_rounds', 'local_lag', 'local_big', 'local_markers', 'local_reconnect', 'scenarios', 'markers',
        'wide', 'synth_c1')


def main():
    subprocess.check_call([sys.executable, os.path.join(REPO, 'oracle/tsref/build_ref.py')])
    replay = os.path.join(REPO, 'oracle/tsref/replay_ref.js')
    spec = spec_docs()
    spec.save(os.path.join(HERE, 'seqdelta.mtlog'))
    print('seqdelta', spec.n_docs, 'docs', spec.n_ops, 'records')
    out = []
    for name in ('seqdelta',) + LOGS:
        res = subprocess.run(['node', replay, 'seqdelta', os.path.join(HERE, name + '.mtlog')], check=True,
                             capture_output=True, text=True)
        for line in res.stdout.strip().split('\n'):
            r = json.loads(line)
            assert r['err'] is None, (name, r['doc'], r['err'])
            ev = r['events']
            row = dict(log=name, doc=r['doc'], err=r['err'], n=len(ev))
            if name == 'seqdelta' or r['doc'] < FULL_DOCS:
                row['events'] = ev
            else:
                row['sha256'] = hashlib.sha256(json.dumps(ev, separators=(',', ':')).encode()).hexdigest()
            out.append(json.dumps(row, separators=(',', ':')))
    with open(os.path.join(HERE, 'seqdelta.expected.jsonl'), 'w') as f:
        f.write('\n'.join(out) + '\n')
    print(len(out), 'rows', os.path.getsize(os.path.join(HERE, 'seqdelta.expected.jsonl')), 'B')


if __name__ == '__main__':
    main()
