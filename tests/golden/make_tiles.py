#!/usr/bin/env python3
"""Regenerate tests/golden/tiles.expected.jsonl FROM THE REFERENCE ITSELF (build container only).

Client.findTile(startPos, tileLabel, preceding) (client.ts:1073-1076 -> mergeTree.ts:1763-1789:
search / backwardSearch with the HierMergeBlock rightmostTiles / leftmostTiles caches) asked of the
reference's own observer Client after each document's log.  Tile labels ride on property key 0:
value id v is the label array ["L<i>" for each bit i of v] under "referenceTileLabels"
(mergeTree.ts:575; js/mtlog.js tileLabels).
  * tiles_scenarios: the findTile cases of client.spec.ts:28-210 restated as remote inserts
    (label "EOP" -> "L0"), plus removed / re-annotated tiles;
  * tiles_synth: marker-heavy synthetic logs (refTypes Tile / NestBegin / NestEnd, labels set at
    insert, tiles removed and zambonied; no annotates, see synthetic()).
One JSON line per (log, document): {log, doc, err, len, answers: [[pos, label, preceding, tile pos |
null], ...]}.  stacks.expected.jsonl: Client.getStackContext(pos, [label]) (client.ts:946-948,
mergeTree.ts:1750-1760) on the same logs with range labels on key 1 ("referenceRangeLabels"):
[[pos, label, [[marker position, refType], ...]], ...].
"""
import json
import os

import numpy as np
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
sys.path.insert(0, HERE)

from fluidframework_amd.oplog import REF_NEST_BEGIN, REF_NEST_END, REF_TILE  # noqa: E402
from make_golden import A, I, M, N, R, build_log  # noqa: E402
from oracle import oracle  # noqa: E402

TILE_KEY = 0
RANGE_KEY = 1


def scenarios():
    docs = []
    L0 = {TILE_KEY: 1}
    # client.spec.ts:29-52: tile at 0, then "abc" at 0 -> tile at 3
    docs.append([M(1, 0, 0, 1, 0, REF_TILE, L0), I(2, 1, 0, 1, 0, 'abc')])
    # :54-75: "abc d", tile at 0
    docs.append([I(1, 0, 0, 1, 0, 'abc d'), M(2, 1, 0, 1, 0, REF_TILE, L0)])
    # :77-149: tile, "abc d" at 0, tile at 0, "ef" at 7, tile at 8
    docs.append([M(1, 0, 0, 1, 0, REF_TILE, L0), I(2, 1, 0, 1, 0, 'abc d'), M(3, 2, 0, 1, 0, REF_TILE, L0),
                 I(4, 3, 0, 1, 7, 'ef'), M(5, 4, 0, 1, 8, REF_TILE, L0)])
    # :151-177: a single tile
    docs.append([M(1, 0, 0, 1, 0, REF_TILE, L0)])
    # :179-203: tile then "abc" before it; index past the end
    docs.append([M(1, 0, 0, 1, 0, REF_TILE, L0), I(2, 1, 0, 1, 0, 'abc')])
    # :205-: text without any tile
    docs.append([I(1, 0, 0, 1, 0, 'abc')])
    # removed tiles (a removed tile is only found as the leaf a backward search stops on), a
    # NestBegin marker with labels (not a Tile), labels rewritten by annotate, an empty document
    docs.append([I(1, 0, 0, 1, 0, 'hello world'), M(2, 1, 0, 2, 5, REF_TILE, {TILE_KEY: 3}),
                 M(3, 2, 0, 1, 8, REF_NEST_BEGIN, {TILE_KEY: 1}), M(4, 3, 0, 2, 12, REF_TILE, {TILE_KEY: 2}),
                 R(5, 4, 0, 1, 5, 6), A(6, 5, 0, 2, 0, 13, {TILE_KEY: 4}), M(7, 6, 0, 3, 13, REF_TILE, L0),
                 R(8, 7, 0, 2, 13, 14)])
    docs.append([I(1, 0, 0, 1, 0, 'ab'), R(2, 1, 0, 1, 0, 2)])
    # many tiles through block splits, then zamboni (msn advance)
    d, s = [], 0
    for k in range(24):
        s += 1
        d.append(M(s, s - 1, 0, 1 + k % 3, k, REF_TILE, {TILE_KEY: 1 + k % 7}) if k % 2 == 0
                 else I(s, s - 1, 0, 1 + k % 3, k, 'p%d' % k))
    s += 1
    d.append(R(s, s - 1, 0, 2, 10, 20))
    for _ in range(4):
        s += 1
        d.append(N(s, s - 1))
    docs.append(d)
    # range stacks (key 1 = "referenceRangeLabels"): nested NestBegin / NestEnd pairs with mixed
    # labels, an unmatched end, a removed begin
    R1 = RANGE_KEY
    docs.append([I(1, 0, 0, 1, 0, 'abcdefghij'), M(2, 1, 0, 1, 1, REF_NEST_BEGIN, {R1: 1}),
                 M(3, 2, 0, 1, 3, REF_NEST_BEGIN, {R1: 3}), M(4, 3, 0, 2, 6, REF_NEST_END, {R1: 2}),
                 M(5, 4, 0, 1, 8, REF_NEST_END, {R1: 1}), M(6, 5, 0, 2, 10, REF_NEST_END, {R1: 1}),
                 M(7, 6, 0, 3, 12, REF_NEST_BEGIN, {R1: 6}), R(8, 7, 0, 1, 3, 4), M(9, 8, 0, 2, 14, REF_TILE, {R1: 1})])
    return build_log(docs)


def synthetic():
    # inserts and removes only: an annotate that changes a tile's labels leaves the reference's
    # HierMergeBlock tile caches stale (annotateRange refreshes no block, mergeTree.ts:2584), which
    # the engine does not reproduce (DESIGN.md "findTile")
    return oracle.generate(16, seed=404, n_clients=10, ops_per_doc=500, max_lag=24, n_keys=2, n_values=15,
                           p_insert=0.6, p_remove=0.4, p_overlap=0.4, p_insert_props=0.6, p_marker=0.4)


def annotated():
    """label annotates between structural changes: an annotate that changes a marker's tile / range
    labels refreshes no block (annotateRange, mergeTree.ts:2565-2605), so the reference answers from
    the labels a block's caches were last rebuilt with until an insert, split, remove, scour, pack or
    ack rebuilds that block (mergeTree.ts:2748-2768)"""
    docs = []
    # ten tiles (labels L0 = 1) with text between them, three leaf blocks; then the middle tiles'
    # labels change to L1 (2) while the blocks stay as they are, and queries from the last block
    # shift over the first ones
    d, s = [], 0
    for k in range(10):
        s += 1
        d.append(M(s, s - 1, 0, 1, 2 * k, REF_TILE, {TILE_KEY: 1}))
        s += 1
        d.append(I(s, s - 1, 0, 1, 2 * k + 1, 'x'))
    for a in (4, 8, 12):
        s += 1
        d.append(A(s, s - 1, 0, 2, a, a + 1, {TILE_KEY: 2}))
    docs.append(d)
    # the same, then an insert into the first block rebuilds it (and only it)
    docs.append(d + [I(s + 1, s, 0, 3, 1, 'ins')])
    # a remove in the middle block rebuilds every block it enters
    docs.append(d + [R(s + 1, s, 0, 3, 9, 10)])
    # range markers: begins labelled R0 (1) re-annotated to R1 (2) and an end gaining R0
    R1 = RANGE_KEY
    d2, s = [], 0
    for k in range(12):
        s += 1
        d2.append(M(s, s - 1, 0, 1, 2 * k, REF_NEST_BEGIN if k % 3 else REF_NEST_END, {R1: 1 if k % 3 else 2}))
        s += 1
        d2.append(I(s, s - 1, 0, 1, 2 * k + 1, 'y'))
    for a, v in ((2, 2), (6, 1), (14, 2)):
        s += 1
        d2.append(A(s, s - 1, 0, 2, a, a + 1, {R1: v}))
    docs.append(d2)
    docs.append(d2 + [N(s + 1, s), N(s + 2, s + 1)])
    hand = build_log(docs)
    synth = oracle.generate(20, seed=606, n_clients=8, ops_per_doc=400, max_lag=16, n_keys=2, n_values=15,
                            p_insert=0.5, p_remove=0.2, p_overlap=0.3, p_null=0.1, p_rewrite=0.05,
                            p_insert_props=0.7, p_marker=0.45)
    return _concat(hand, synth)


def _concat(a, b):
    """one log holding a's documents, then b's"""
    from fluidframework_amd.oplog import OpBatch
    ops_b = b.ops.copy()
    ops_b['payload_off'] += len(a.payload)
    return OpBatch(np.concatenate([a.ops, ops_b]), np.concatenate([a.payload, b.payload]),
                   np.concatenate([a.row_ptr, b.row_ptr[1:] + a.row_ptr[-1]]).astype(np.uint32))


def main():
    subprocess.check_call([sys.executable, os.path.join(REPO, 'oracle/tsref/build_ref.py')])
    oracle.build()
    replay = os.path.join(REPO, 'oracle/tsref/replay_ref.js')
    out = []
    for name, batch in (('tiles_scenarios', scenarios()), ('tiles_synth', synthetic()), ('tiles_annot', annotated())):
        path = os.path.join(HERE, name + '.mtlog')
        batch.save(path)
        res = subprocess.run(['node', replay, 'tiles', path, str(TILE_KEY)], check=True, capture_output=True,
                             text=True)
        for line in res.stdout.strip().split('\n'):
            r = json.loads(line)
            out.append(json.dumps(dict(log=name, **r), separators=(',', ':')))
        print(name, batch.n_docs, 'docs')
    with open(os.path.join(HERE, 'tiles.expected.jsonl'), 'w') as f:
        f.write('\n'.join(out) + '\n')
    # getStackContext on the same logs, range labels on key 1
    out = []
    for name in ('tiles_scenarios', 'tiles_synth', 'tiles_annot'):
        res = subprocess.run(['node', replay, 'stacks', os.path.join(HERE, name + '.mtlog'), str(RANGE_KEY)],
                             check=True, capture_output=True, text=True)
        for line in res.stdout.strip().split('\n'):
            r = json.loads(line)
            out.append(json.dumps(dict(log=name, **r), separators=(',', ':')))
    with open(os.path.join(HERE, 'stacks.expected.jsonl'), 'w') as f:
        f.write('\n'.join(out) + '\n')


if __name__ == '__main__':
    main()
