"""Delta / maintenance events of the batched engine (include/mtgpu.h "delta / maintenance events").

The reference fires `Client.mergeTreeDeltaCallback(opArgs, {operation, deltaSegments})` and
`mergeTreeMaintenanceCallback({operation, deltaSegments})` synchronously inside `applyMsg`
(packages/dds/merge-tree/src/mergeTreeDeltaCallback.ts:15-73; fired at mergeTree.ts:1981-1988,
2231-2236, 1310-1315, 1335-1340, 2592-2600, 2705-2712).  The engine records them per document as
`mt_event` rows (one per delta segment); this module groups the rows back into callbacks.

Canonical callback form (what tests compare, and what oracle/tsref/replay_ref.js writes from the
reference's own callbacks): ``[seq, operation, [[leaf, pos, len, propertyDeltas], ...]]`` with
operation = MergeTreeDeltaType (INSERT 0, REMOVE 1, ANNOTATE 2) or MergeTreeMaintenanceType (APPEND
-1, SPLIT -2, UNLINK -3); propertyDeltas = ``{"k<id>": previous value id | None}`` for ANNOTATE
(sorted keys), else None.
"""
import numpy as np

EVENT_DTYPE = np.dtype([('seq', '<i4'), ('op', 'i1'), ('flags', 'u1'), ('pad', '<u2'), ('leaf', '<i4'),
                        ('pos', '<i4'), ('len', '<u4'), ('pmask', '<u4'), ('pvals', '<u2', (32,)), ('pad2', '<u8')])
assert EVENT_DTYPE.itemsize == 96

EV_INSERT, EV_REMOVE, EV_ANNOTATE = 0, 1, 2
EV_APPEND, EV_SPLIT, EV_UNLINK = -1, -2, -3
EVF_FIRST, EVF_EMPTY, EVF_NOPD = 1, 2, 4
OP_NAMES = {EV_INSERT: 'INSERT', EV_REMOVE: 'REMOVE', EV_ANNOTATE: 'ANNOTATE', EV_APPEND: 'APPEND',
            EV_SPLIT: 'SPLIT', EV_UNLINK: 'UNLINK'}


def property_deltas(pmask, pvals):
    """propertyDeltas of an ANNOTATE record: {"k<id>": previous value id, or None (null)}."""
    out = {}
    for k in range(32):
        if (pmask >> k) & 1:
            v = int(pvals[k])
            out['k%d' % k] = v if v else None
    return out


def callbacks(rows):
    """Group one document's mt_event rows into canonical callbacks (module docstring)."""
    out = []
    for r in rows:
        op = int(r['op'])
        flags = int(r['flags'])
        if flags & EVF_FIRST:
            out.append([int(r['seq']), op, []])
        if not out:
            raise ValueError('event stream does not start with a callback')
        if flags & EVF_EMPTY:
            continue
        pd = property_deltas(int(r['pmask']), r['pvals']) if op == EV_ANNOTATE and not flags & EVF_NOPD else None
        out[-1][2].append([int(r['leaf']), int(r['pos']), int(r['len']), pd])
    return out
