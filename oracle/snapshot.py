"""CPU restatement of SnapshotV1 extraction + emit -- TEST INFRASTRUCTURE
ONLY (the checker of the engine's mt_get_snapshot; imported by tests/ only).

Input: a document's canonical state (oracle.Oracle.state(d) / mt_get_state: L2 linked leaves in
order, currentSeq, minSeq).  Follows:

  SnapshotV1.extractSync  packages/dds/merge-tree/src/snapshotV1.ts:151-247
  SnapshotV1.emit          snapshotV1.ts:85-149, getSeqLengthSegs :57-79
  TextSegment.canAppend / append / toJSONObject  textSegment.ts:47-85
  matchProperties          properties.ts:62-93 (on interned value ids: map equality, and a
                           defined-but-empty map differs from undefined)

Pinned by tests/golden/*.snapshot*.jsonl, written by the reference itself (make_snapshots.py).
"""
TEXT_GRANULARITY = 256          # MergeTree.TextSegmentGranularity (mergeTree.ts:1059)
DEFAULT_CHUNK = 10000           # SnapshotV1.chunkSize (snapshotV1.ts:40)


def client_name(c):
    return 'observer' if c == 0 else 'c%d' % c


def _json(text, props):
    if isinstance(text, dict):                       # Marker.toJSONObject (mergeTree.ts:652-656)
        spec = {'marker': {'refType': text['marker']}}
        if props is not None:
            spec['props'] = props
        return spec
    return text if props is None else {'text': text, 'props': props}       # toJSONObject


def extract(state, name=client_name):
    """extractSync: the segment specs and their lengths."""
    msn = state['msn']
    specs, lens = [], []
    prev = None                                      # [text, props] of the coalescing candidate

    def push(p):
        specs.append(_json(p[0], p[1]))
        lens.append(1 if isinstance(p[0], dict) else len(p[0]))

    for text, seq, c, rseq, rc, _ov, props in state['segs']:
        removed = rseq != -1 or rc != -1             # (a pending local removal: rseq -1 by the editing client)
        if seq == -1:                                # a pending local insert: elided (snapshotV1.ts:184)
            continue
        if removed and rseq <= msn:                  # removed at or below the MSN (or pending): elided
            continue
        if seq <= msn and not removed:               # below the MSN: coalesce
            mk = isinstance(text, dict) or (prev is not None and isinstance(prev[0], dict))
            if prev is None:
                prev = [text, props]
            elif (not mk and not prev[0].endswith('\n')       # canAppend: text segments only
                  and (len(prev[0]) <= TEXT_GRANULARITY or len(text) <= TEXT_GRANULARITY) and prev[1] == props):
                prev[0] += text                      # clone + append
            else:
                push(prev)
                prev = [text, props]
        else:                                        # keeps its merge info
            if prev is not None:
                push(prev)
            prev = None
            raw = {'json': _json(text, props)}
            if seq > msn:
                raw['seq'] = seq
                raw['client'] = name(c)
            if removed:
                raw['removedSeq'] = rseq
                raw['removedClient'] = name(rc)
            specs.append(raw)
            lens.append(1 if isinstance(text, dict) else len(text))
    if prev is not None:
        push(prev)
    return specs, lens


def emit(state, chunk=DEFAULT_CHUNK, name=client_name):
    """emit(): tree entries path -> parsed blob contents (header + body_i)."""
    specs, lens = extract(state, name)
    chunks, count, total = [], 0, 0
    while True:
        start, length, n = count, 0, 0
        while length < chunk and start + n < len(specs):
            length += lens[start + n]
            n += 1
        chunks.append({'version': '1', 'segmentCount': n, 'length': length, 'segments': specs[start:start + n],
                       'startIndex': start})
        count += n
        total += length
        if not count < len(specs):
            break
    header = chunks[0]
    header['headerMetadata'] = {
        'minSequenceNumber': state['msn'], 'sequenceNumber': state['seq'],
        'orderedChunkMetadata': [{'id': 'header'}] + [{'id': 'body_%d' % i} for i in range(len(chunks) - 1)],
        'totalLength': total, 'totalSegmentCount': count}
    out = {'header': header}
    for i, ch in enumerate(chunks[1:]):
        out['body_%d' % i] = ch
    return out
