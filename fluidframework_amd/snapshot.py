"""Snapshot load on the host side of the engine: the reference's SnapshotLoader
(packages/dds/merge-tree/src/snapshotLoader.ts:24-253) for many documents at once.

A merge-tree snapshot is a tree of blobs: the header chunk (snapshotLegacy.ts:45-47 `header`) and,
for long documents, body chunks (`body_0`.. in v1, `body` in the legacy format), plus an optional
`catchupOps` blob (legacy).  The chunks are parsed and brought to the v1 shape exactly as
toLatestVersion does (snapshotChunks.ts:133-185); then

  * the header's segments become the document through mt_docs_load -- reloadFromSegments
    (mergeTree.ts:1195-1251) + startOrUpdateCollaboration(minSeq, seq) on the device;
  * every body segment becomes an MT_OP_LOAD record, applied by the engine's own insert path as
    loadBody's insertSegments(root.cachedLength, ...) (snapshotLoader.ts:192-224) does;
  * catch-up ops are returned to the caller, to be submitted like any other sequenced ops.

Segment specs (IJSONSegment / IJSONSegmentWithMergeInfo, snapshotChunks.ts:60-73) map as
SnapshotLoader.specToSegment (snapshotLoader.ts:85-117) does: without merge info a segment is
(UniversalSequenceNumber 0, NonCollabClient); with it, its seq / client / removedSeq / removedClient.
Long client ids and property keys / values are interned per document by the caller's interners.
Marker specs ({marker: {refType}, props}, Marker.toJSONObject mergeTree.ts:652-656) load as markers
(one byte, the ReferenceType, up to 255).  Text is carried as UTF-16 code units (cachedLength =
text.length, textSegment.ts:45): Latin-1 bytes when every unit fits, else 2 bytes per unit
(MT_LSF_U16; the document loads in the engine's wide form, include/mtgpu.h "limits"), as are keys
>= 8, value ids >= 256 and client ids >= 64.
"""
import ctypes
import json

import numpy as np

from .engine import _check, _ptr, lib
from .oplog import F_MARKER, F_PROPS, OP_DTYPE, OP_WIDE, OpBatch, encode_text, pack_npairs

MT_OP_LOAD = 4
NONCOLLAB = 0xFE            # MT_CLIENT_NONCOLLAB: NonCollabClient (constants.ts:15)
UNIVERSAL_SEQ = 0           # UniversalSequenceNumber (constants.ts:11)
SF_PDEF = 2
SF_MARKER = 16
LSF_U16 = 64                # MT_LSF_U16: the segment's text is UTF-16 code units

LOAD_SEG_DTYPE = np.dtype([('seq', '<i4'), ('rseq', '<i4'), ('client', 'u1'), ('rclient', 'u1'), ('flags', 'u1'),
                           ('pad', 'u1'), ('text_off', '<u4'), ('text_len', '<u4'), ('client_hi', 'u1'),
                           ('rclient_hi', 'u1'), ('pad2', '<u2'),
                           ('props', '<u2', (32,)), ('pad3', '<u8')])
assert LOAD_SEG_DTYPE.itemsize == 96


class Interner:
    """First-appearance ids (Client.getOrAddShortClientId order, client.ts:636-660); `first` is the
    first id handed out (1 for clients: 0 is the document's own observer)."""

    def __init__(self, first=1, limit=64):
        self.ids = {}
        self.first, self.limit = first, limit

    def __call__(self, key):
        k = json.dumps(key, sort_keys=True)  # (a value "true" and a value true are different ids)
        if k not in self.ids:
            if self.first + len(self.ids) >= self.limit:
                raise ValueError(f'more than {self.limit - self.first} distinct ids in one document')
            self.ids[k] = self.first + len(self.ids)
        return self.ids[k]


class ClientInterner(Interner):
    """Short client ids 1..65534 in first-appearance order, skipping 254 (NonCollabClient's:
    include/mtgpu.h MT_CLIENT_NONCOLLAB; ids from 64 on make the document wide)."""

    def __init__(self):
        super().__init__(1, 65535)

    def __call__(self, key):
        k = json.dumps(key, sort_keys=True)
        if k not in self.ids:
            n = self.first + len(self.ids)
            n += 1 if n >= NONCOLLAB else 0
            if n >= self.limit:
                raise ValueError(f'more than {self.limit - 2} distinct client ids in one document')
            self.ids[k] = n
        return self.ids[k]


class DocInterners:
    """Per-document id spaces: long client ids -> short ids (1..65534 but 254), property keys ->
    0..31, and per key its values -> 1..65535 (0 = absent; ids are opaque, only equality matters,
    properties.ts:62-93)."""

    def __init__(self):
        self.client = ClientInterner()
        self.key = Interner(0, 32)
        self.values = {}

    def value(self, kid, v):
        if kid not in self.values:
            self.values[kid] = Interner(1, 65536)
        return self.values[kid](v)


def _blobs(tree):
    """{path: contents str or parsed} of a snapshot: an ITree ({"entries": [...]}, e.g. the
    reference's sequence/src/test/snapshots/*.json; a SharedString keeps the merge-tree under
    "content"), or the {path: parsed chunk} form mt_get_snapshot / SnapshotV1.emit produce."""
    if isinstance(tree, dict) and 'entries' in tree:
        entries = tree['entries']
        content = [e for e in entries if e.get('path') == 'content' and e.get('type') == 'Tree']
        if content:
            entries = content[0]['value']['entries']
        return {e['path']: e['value']['contents'] for e in entries if e.get('type') == 'Blob'}
    return dict(tree)


def _parse(x):
    return json.loads(x) if isinstance(x, str) else x


def to_latest_version(path, chunk):
    """snapshotChunks.ts:133-185: a legacy chunk (version undefined) in the v1 shape."""
    if chunk.get('version') == '1':
        return chunk
    if chunk.get('version') is not None:
        raise ValueError(f'Unsupported chunk path: {path} version: {chunk.get("version")}')
    meta = None
    if path == 'header':
        meta = chunk.get('headerMetadata')
        if meta is None:
            ids = [{'id': 'header'}]
            if chunk['chunkLengthChars'] < chunk['totalLengthChars']:
                ids.append({'id': 'body'})
            meta = {'orderedChunkMetadata': ids, 'minSequenceNumber': chunk.get('chunkMinSequenceNumber'),
                    'sequenceNumber': chunk.get('chunkSequenceNumber'), 'totalLength': chunk['totalLengthChars'],
                    'totalSegmentCount': chunk['totalSegmentCount']}
    return {'version': '1', 'length': chunk['chunkLengthChars'], 'segmentCount': chunk['chunkSegmentCount'],
            'headerMetadata': meta, 'segments': chunk['segmentTexts'], 'startIndex': chunk['chunkStartSegmentIndex']}


class LoadedDoc:
    """One document's snapshot, parsed: header specs, body specs, window, catch-up ops."""

    def __init__(self, tree):
        blobs = _blobs(tree)
        header = to_latest_version('header', _parse(blobs['header']))
        meta = header.get('headerMetadata')
        if meta is None:
            raise ValueError('header metadata not available')
        # snapshotLoader.ts:159-190: every further chunk in orderedChunkMetadata order
        self.header = list(header['segments'])
        self.body = []
        if header['segmentCount'] != meta['totalSegmentCount']:
            for md in meta['orderedChunkMetadata'][1:]:
                self.body.extend(to_latest_version(md['id'], _parse(blobs[md['id']]))['segments'])
        known = {md['id'] for md in meta['orderedChunkMetadata']}
        rest = [p for p in blobs if p not in known]
        self.catchup = _parse(blobs[rest[0]]) if len(rest) == 1 and blobs[rest[0]] else []
        if len(rest) > 1:
            raise ValueError('Unexpected blobs in snapshot')
        self.seq = meta['sequenceNumber']
        self.min_seq = meta['minSequenceNumber'] if meta.get('minSequenceNumber') is not None else self.seq


def _spec(spec, it):
    """specToSegment (snapshotLoader.ts:85-117) -> (text, seq, client, rseq, rclient, pdef, props
    {key id: value id}, marker)"""
    merge = isinstance(spec, dict) and 'json' in spec
    js = spec['json'] if merge else spec
    marker = False
    if isinstance(js, str):
        text, props = js, None
    elif isinstance(js, dict) and 'text' in js:
        text, props = js['text'], js.get('props')
    elif isinstance(js, dict) and 'marker' in js:    # Marker.fromJSONObject (mergeTree.ts:658-665)
        rt = js['marker'].get('refType', 0)
        if not 0 <= rt <= 255:
            raise ValueError(f'marker refType {rt} is not device-representable')
        text, props, marker = chr(rt), js.get('props'), True
    else:
        raise ValueError(f'not a text or marker segment spec: {json.dumps(js)[:80]}')
    pv = {}
    if props is not None:
        for k, v in props.items():
            if v is None:  # a null value never reaches a stored property set
                continue
            kid = it.key(k)
            pv[kid] = it.value(kid, v)
    if merge:
        seq = spec['seq'] if spec.get('seq') is not None else UNIVERSAL_SEQ
        client = it.client(spec['client']) if spec.get('client') is not None else NONCOLLAB
        rseq = spec['removedSeq'] if spec.get('removedSeq') is not None else -1
        rclient = it.client(spec['removedClient']) if spec.get('removedClient') is not None else 0
    else:
        seq, client, rseq, rclient = UNIVERSAL_SEQ, NONCOLLAB, -1, 0
    return text, seq, client, rseq, rclient, props is not None, pv, marker


def _wide_seg(units_wide, client, rseq, rclient, pv):
    return (units_wide or (client >= 64 and client != NONCOLLAB) or (rseq >= 0 and rclient >= 64) or
            any(k >= 8 or v > 255 for k, v in pv.items()))


def build_load(docs, interners=None):
    """Device inputs for a batch of parsed documents: (segs, text, row_ptr, min_seq, cur_seq,
    body OpBatch of MT_OP_LOAD records, interners)."""
    interners = interners or [DocInterners() for _ in docs]
    segs, text, row_ptr = [], bytearray(), [0]
    recs, payload, body_rp = [], bytearray(), [0]
    for doc, it in zip(docs, interners):
        local = 0  # root.cachedLength: the local (non-removed) length
        for spec in doc.header:
            t, seq, client, rseq, rclient, pdef, pv, mk = _spec(spec, it)
            tb, wide_text = encode_text(t)
            n = len(tb) // 2 if wide_text else len(tb)
            props = [pv.get(k, 0) for k in range(32)]
            rc = rclient if rseq >= 0 else 0
            segs.append((seq, rseq, client & 0xFF, rc & 0xFF,
                         (SF_PDEF if pdef else 0) | (SF_MARKER if mk else 0) | (LSF_U16 if wide_text else 0), 0,
                         len(text), n, client >> 8, rc >> 8, 0, props, 0))
            text += tb
            local += 0 if rseq >= 0 else n
        row_ptr.append(len(segs))
        # loadBody (snapshotLoader.ts:192-224): a run of segments without merge info is one
        # insertSegments at root.cachedLength, each next one at insertPos += cachedLength
        # (mergeTree.ts:2219); any other segment is its own insertSegments call
        batch_pos = None
        for spec in doc.body:
            t, seq, client, rseq, rclient, pdef, pv, mk = _spec(spec, it)
            tb, wide_text = encode_text(t)
            n = len(tb) // 2 if wide_text else len(tb)
            wide = _wide_seg(wide_text, client, rseq, rclient, pv)
            if wide and not wide_text:  # a wide record carries its text as UTF-16 units
                tb, wide_text = encode_text(t, force_wide=True)
            batched = client == NONCOLLAB and seq == UNIVERSAL_SEQ
            if batched:
                pos = local if batch_pos is None else batch_pos
                batch_pos = pos + n
            else:
                pos = local
                batch_pos = None
            local += 0 if rseq >= 0 else n
            pairs = b''
            flags = tbits = 0
            if pdef:
                for k in sorted(pv):
                    pairs += bytes([k, pv[k] & 0xFF, pv[k] >> 8]) if wide else bytes([k, pv[k]])
                fbits, tbits = pack_npairs(len(pv), wide)
                flags = F_PROPS | fbits
            if mk:
                flags |= F_MARKER
            data = tb + pairs
            rc = rclient if rseq >= 0 else 0
            # (MT_OP_LOAD: the ids' low bytes in `client`, their high bytes in `msn`)
            recs.append((seq, UNIVERSAL_SEQ, (client >> 8) | ((rc >> 8) << 8), (client & 0xFF) | ((rc & 0xFF) << 8),
                         MT_OP_LOAD | (OP_WIDE if wide else 0) | tbits, flags, pos, rseq, len(payload), len(data)))
            payload += data
        body_rp.append(len(recs))
    segs_a = np.array(segs, dtype=LOAD_SEG_DTYPE) if segs else np.zeros(0, dtype=LOAD_SEG_DTYPE)
    body = OpBatch(np.array(recs, dtype=OP_DTYPE) if recs else np.zeros(0, dtype=OP_DTYPE),
                   np.frombuffer(bytes(payload), dtype=np.uint8).copy(), np.array(body_rp, dtype=np.uint32))
    return (segs_a, np.frombuffer(bytes(text), dtype=np.uint8).copy(), np.array(row_ptr, dtype=np.uint32),
            np.array([d.min_seq for d in docs], dtype=np.int32), np.array([d.seq for d in docs], dtype=np.int32),
            body, interners)


def load_docs(engine, trees, doc_ids=None, interners=None):
    """Load one snapshot per document into `engine` (documents doc_ids, default 0..n-1): the
    header through mt_docs_load, then the body appends through the engine's apply (documents
    without a snapshot in the batch get no ops).  Returns (interners, catch-up ops per doc)."""
    return load_parsed(engine, [LoadedDoc(t) for t in trees], doc_ids, interners)


def load_parsed(engine, docs, doc_ids=None, interners=None):
    """load_docs for documents already parsed: objects with LoadedDoc's fields (header and body
    specs, seq, min_seq, catchup)."""
    ids = np.arange(len(docs), dtype=np.uint32) if doc_ids is None else np.ascontiguousarray(doc_ids, np.uint32)
    segs, text, rp, mn, cs, body, its = build_load(docs, interners)
    L = lib()
    L.mt_docs_load.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                               ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p]
    L.mt_docs_load.restype = ctypes.c_int
    _check(L.mt_docs_load(engine.h, len(docs), _ptr(ids), _ptr(rp), _ptr(segs), _ptr(text), len(text), _ptr(mn),
                          _ptr(cs)), 'mt_docs_load')
    if body.n_ops:
        # the engine applies a batch over all its documents: scatter the body rows to doc_ids
        counts = np.zeros(engine.n_docs, dtype=np.int64)
        counts[ids] = np.diff(body.row_ptr)
        row_ptr = np.zeros(engine.n_docs + 1, dtype=np.uint32)
        row_ptr[1:] = np.cumsum(counts)
        order = np.argsort(ids, kind='stable')
        ops = np.concatenate([body.ops[body.row_ptr[i]:body.row_ptr[i + 1]] for i in order]) if len(order) else body.ops
        engine.apply(OpBatch(ops, body.payload, row_ptr))
    return its, [d.catchup for d in docs]
