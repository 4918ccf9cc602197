#!/usr/bin/env python3
"""Golden fixtures beyond the narrow device limits (include/mtgpu.h "limits") FROM THE REFERENCE ITSELF.

Runs in the build container only (needs /root/reference and node): op logs are written, then
oracle/tsref/replay_ref.js replays each through the reference observer Client and its canonical state
is stored as the expected output (the make_golden.py pattern).
  * wide.mtlog / wide.expected.jsonl -- hand-made scenarios: CJK text split mid-run, surrogate pairs
    split by inserts and removes and rejoined by zamboni, 120 client ids with eight overlapping
    removers >= 64 on one segment, value ids up to 65535 and keys 8..15 (annotate, rewrite, null),
    a narrow document promoted mid-life by a wide op and by a client id >= 64, markers with wide props;
  * wide_synth.mtlog / .expected.jsonl -- observer-driven logs over the reference
    (oracle/tsref/wide_log.js): 120 clients per document, UTF-16 text with CJK and surrogate pairs,
    value ids past 255, keys past 7;
  * wide_many.mtlog / .expected.jsonl -- short client ids past 255 (320 clients per document) and
    sixteen overlapping removers >= 64 on one segment (hand-made), plus wide_log.js documents with
    320 clients;
  * wide_xl.mtlog / .expected.jsonl -- past sixteen: twenty and thirty-two overlapping removers >= 64
    on one segment, records with 24 and 32 property keys (MT_OP_NP32), keys 16..31 on markers, plus
    wide_log.js documents drawing from 32 keys.
Fixtures are data only (inputs and reference outputs).
"""
import json
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
sys.path.insert(0, HERE)

from make_golden import A, I, M, N, R, build_log  # noqa: E402
from fluidframework_amd.oplog import REF_TILE  # noqa: E402
from oracle import canon  # noqa: E402


def scenarios():
    docs = []
    # 0: CJK text, an insert splitting it, a remove across the split, an annotate with a wide value,
    #    then the msn passes everything (zamboni appends the CJK runs back together)
    docs.append([I(1, 0, 0, 1, 0, '中文字符串'), I(2, 1, 0, 2, 2, 'ab'), R(3, 2, 1, 3, 1, 4), A(4, 3, 2, 1, 0, 3, {0: 300}),
                 I(5, 4, 3, 2, 4, '漢'), N(6, 5), N(7, 6)])
    # 1: surrogate pairs: an insert between the halves of one, a remove of half of another, a split
    #    by an annotate boundary; zamboni rejoins the halves
    docs.append([I(1, 0, 0, 1, 0, 'a😀b🎉c'), I(2, 1, 0, 2, 2, 'X'), R(3, 2, 1, 3, 5, 7), A(4, 3, 2, 1, 1, 2, {1: 7}),
                 I(5, 2, 2, 3, 1, '𝄞'), N(6, 5), N(7, 6), N(8, 7)])
    # 2: 120 client ids: every client inserts once, then client 65 removes a range and clients
    #    66..73 remove it concurrently (eight overlapping removers >= 64, the wide form's list), and
    #    later clients see the removal
    d, s = [], 0
    for k in range(1, 121):
        s += 1
        d.append(I(s, s - 1, 0, k, 0, chr(ord('a') + k % 26)))
    base = s
    for j, k in enumerate(range(65, 74)):
        s += 1
        d.append(R(s, base, 0, k, 2, 9 + j % 3))
    s += 1
    d.append(I(s, s - 1, 0, 110, 3, 'late'))
    s += 1
    d.append(R(s, base, 0, 40, 3, 6))   # a narrow overlapper too
    for _ in range(3):  # (the msn stays below the removals: the overlap sets survive in the final state)
        s += 1
        d.append(N(s, base - 4))
    docs.append(d)
    # 3: keys 8..15 and value ids up to 65535: set, rewrite, null delete, merge back by zamboni
    docs.append([I(1, 0, 0, 1, 0, 'hello world', {9: 65535}), A(2, 1, 0, 2, 0, 5, {15: 4000, 3: 256}),
                 A(3, 2, 0, 3, 3, 8, {9: None, 12: 70}), A(4, 3, 0, 2, 1, 4, {8: 1}, flags=1), I(5, 4, 0, 1, 11, '!'),
                 A(6, 5, 0, 4, 0, 12, {3: 256}), N(7, 6), N(8, 7)])
    # 4: a narrow document (Latin-1, clients < 64, an overlap among them) promoted mid-life by a wide
    #    insert; then more narrow ops apply to the wide document
    d = [I(1, 0, 0, 1, 0, 'alpha beta'), I(2, 1, 0, 2, 5, '\n'), R(3, 2, 1, 3, 0, 3), R(4, 2, 1, 4, 1, 4),
         N(5, 3), I(6, 5, 4, 5, 2, 'price: 5€'), A(7, 6, 5, 1, 0, 4, {2: 9}), R(8, 7, 6, 2, 3, 6), N(9, 8), N(10, 9)]
    docs.append(d)
    # 5: promotion by a client id >= 64 whose removal joins a segment's narrow overlap set
    docs.append([I(1, 0, 0, 1, 0, 'abcdefgh'), R(2, 1, 0, 2, 2, 6), R(3, 1, 0, 3, 3, 5), R(4, 1, 0, 100, 2, 7),
                 I(5, 4, 1, 99, 0, 'Z'), N(6, 5), N(7, 6)])
    # 6: markers with wide props among UTF-16 text
    docs.append([I(1, 0, 0, 1, 0, 'x€y'), M(2, 1, 0, 2, 1, REF_TILE, {3: 1000}), M(3, 2, 0, 3, 3, REF_TILE, {10: 2}),
                 A(4, 3, 0, 1, 0, 5, {3: 999}), R(5, 4, 1, 2, 0, 1), N(6, 5), N(7, 6)])
    return build_log(docs)


def many():
    """More client ids than a byte holds and a full overlap list of high ids:
    include/mtgpu.h MT_MAX_CLIENTS_WIDE / MT_OVX_IDS.  Short ids skip 254 (NonCollabClient's)."""
    ids = [k for k in range(1, 330) if k != 254]
    docs = []
    # 0: 320 clients insert once each; then 14 clients with ids >= 256 and two in 64..255 remove one
    #    range concurrently -- sixteen overlapping removers >= 64, the device list full -- plus a
    #    narrow one; later ops by ids past 300 see the removal, an annotate by one splits the range
    d, s = [], 0
    for k in ids[:320]:
        s += 1
        d.append(I(s, s - 1, 0, k, 0, chr(ord('a') + k % 26)))
    base = s
    removers = [100, 300, 256, 257, 258, 259, 260, 261, 262, 263, 264, 265, 266, 267, 268, 200, 40]
    for j, k in enumerate(removers):
        s += 1
        d.append(R(s, base, 0, k, 10, 20 + j % 4))
    s += 1
    d.append(I(s, s - 1, 0, 310, 5, 'after'))
    s += 1
    d.append(A(s, s - 1, 0, 305, 3, 12, {2: 7}))
    for _ in range(3):  # (the msn stays below the removals: the overlap sets survive in the final state)
        s += 1
        d.append(N(s, base - 4))
    docs.append(d)
    # 1: overlapping removes by ids 255..301 interleaved with ids below 256, then the msn passes
    #    everything: zamboni unlinks the removed segments and packs the rest
    d, s = [], 0
    for k in ids[:300]:
        s += 1
        d.append(I(s, s - 1, 0, k, min(s % 7, 2 * (s - 1)), 'xy'))
    base = s
    for j, k in enumerate([255, 70, 299, 301, 280, 65, 290]):
        s += 1
        d.append(R(s, base, 0, k, 20 + j, 40 + j))
    s += 1
    d.append(I(s, base, 0, 302, 30, 'mid'))
    for _ in range(4):
        s += 1
        d.append(N(s, s - 1))
    docs.append(d)
    # 2: records carrying all sixteen keys (a 16-pair record: MT_OP_NP16): an insert with sixteen
    #    props, an annotate setting all sixteen, a rewrite with sixteen (four of them null)
    docs.append([I(1, 0, 0, 1, 0, 'sixteen keys here', {k: 300 + k for k in range(16)}),
                 A(2, 1, 0, 2, 2, 9, {k: 1000 + k for k in range(16)}),
                 A(3, 2, 0, 300, 5, 14, {k: (None if k % 4 == 0 else 2000 + k) for k in range(16)}, flags=1),
                 I(4, 3, 1, 256, 3, 'x', {15: 9}), N(5, 4), N(6, 5)])
    docs += synth_docs(6, 2029, 900, 320, 12)
    return build_log(docs)


def xl():
    """Past sixteen property keys and sixteen overlapping high-id removers:
    include/mtgpu.h MT_MAX_KEYS_WIDE = 32, MT_OVX_IDS = 32 (the reference's maps are unbounded:
    properties.ts:156-170 createMap, mergeTree.ts:2544-2552 addOverlappingClient)."""
    ids = [k for k in range(1, 140) if k != 254]
    docs = []
    # 0: 120 clients insert once each; then 21 clients >= 64 and a narrow one remove one range
    #    concurrently (twenty overlapping removers >= 64 after the first); later ids see the removal
    d, s = [], 0
    for k in ids[:120]:
        s += 1
        d.append(I(s, s - 1, 0, k, 0, chr(ord('a') + k % 26)))
    base = s
    removers = [64 + j for j in range(21)] + [12]
    for j, k in enumerate(removers):
        s += 1
        d.append(R(s, base, 0, k, 10, 24 + j % 5))
    s += 1
    d.append(I(s, s - 1, 0, 119, 5, 'after'))
    s += 1
    d.append(A(s, s - 1, 0, 118, 3, 12, {20: 7}))
    for _ in range(3):  # (the msn stays below the removals: the overlap sets survive in the final state)
        s += 1
        d.append(N(s, base - 4))
    docs.append(d)
    # 1: thirty-three removers >= 64 on one range: the first takes removedClient, thirty-two
    #    overlap it (the device list full); then the msn passes everything and zamboni unlinks them
    d, s = [], 0
    for k in ids[:110]:
        s += 1
        d.append(I(s, s - 1, 0, k, min(s % 5, s - 1), 'pq'))
    base = s
    for j in range(33):
        s += 1
        d.append(R(s, base, 0, 70 + j, 30, 50))
    s += 1
    d.append(I(s, base, 0, 108, 40, 'mid'))
    for _ in range(3):
        s += 1
        d.append(N(s, base - 2))
    s += 1
    d.append(N(s, s - 1))
    docs.append(d)
    # 2: twenty-four keys: an insert with 24 props (keys 0..23), an annotate setting all 32 (a
    #    32-pair record: MT_OP_NP32), a rewrite with 20 (five null), null deletes of keys >= 16,
    #    and segments that differ only in keys >= 16 (zamboni must not merge them)
    docs.append([I(1, 0, 0, 1, 0, 'twenty four keys', {k: 100 + k for k in range(24)}),
                 A(2, 1, 0, 2, 2, 9, {k: 1000 + k for k in range(32)}),
                 A(3, 2, 0, 3, 5, 14, {k: (None if k % 4 == 0 else 2000 + k) for k in range(4, 24)}, flags=1),
                 A(4, 3, 0, 2, 0, 3, {17: None, 23: None, 31: 5}),
                 I(5, 4, 1, 4, 3, 'x', {31: 9}),
                 A(6, 5, 2, 1, 6, 8, {29: 300}),
                 I(7, 6, 3, 5, 0, 'plain'), N(8, 7), N(9, 8)])
    # 3: markers with keys >= 16 among UTF-16 text, and an annotate of keys 16..31 across them
    docs.append([I(1, 0, 0, 1, 0, 'x€y z'), M(2, 1, 0, 2, 1, REF_TILE, {16: 1000, 3: 1}),
                 M(3, 2, 0, 3, 3, REF_TILE, {30: 2}),
                 A(4, 3, 0, 1, 0, 6, {k: 40 + k for k in range(16, 32)}), R(5, 4, 1, 2, 0, 1), N(6, 5), N(7, 6)])
    docs += synth_docs(6, 2031, 800, 140, 10, 32)
    return build_log(docs)


def synth_docs(n_docs, seed, ops, clients, lag=8, keys=16):
    res = subprocess.run(['node', os.path.join(REPO, 'oracle/tsref/wide_log.js'), str(n_docs), str(seed), str(ops),
                          str(clients), str(lag), str(keys)], check=True, capture_output=True, text=True)
    docs = json.loads(res.stdout)['docs']
    out = []
    for d in docs:
        recs = []
        for (seq, ref, msn, c, typ, p1, p2, text, props, flags) in d:
            props = None if props is None else {int(k): v for k, v in props.items()}
            recs.append((seq, ref, msn, c, typ, p1, p2, text, props, flags))
        out.append(recs)
    return out


def synth(n_docs, seed, ops, clients, lag=8):
    return build_log(synth_docs(n_docs, seed, ops, clients, lag))


def main():
    subprocess.check_call([sys.executable, os.path.join(REPO, 'oracle/tsref/build_ref.py')])
    replay = os.path.join(REPO, 'oracle/tsref/replay_ref.js')
    sets = (('wide', scenarios()), ('wide_synth', synth(12, 2027, 700, 120)), ('wide_many', many()),
            ('wide_xl', xl()))
    for name, batch in sets:
        if len(sys.argv) > 1 and name not in sys.argv[1:]:
            continue
        path = os.path.join(HERE, name + '.mtlog')
        batch.save(path)
        res = subprocess.run(['node', replay, 'state', path], check=True, capture_output=True, text=True)
        lines = []
        for line in res.stdout.strip().split('\n'):
            r = json.loads(line)
            r['checksum'] = '%016x' % canon.checksum(r['state'])
            lines.append(json.dumps(r, separators=(',', ':')))
        with open(os.path.join(HERE, name + '.expected.jsonl'), 'w') as f:
            f.write('\n'.join(lines) + '\n')
        print(name, batch.n_docs, 'docs', batch.n_ops, 'ops', os.path.getsize(path), 'B')


if __name__ == '__main__':
    main()
