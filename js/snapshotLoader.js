"use strict";
// snapshotLoader.js -- SnapshotLoader (packages/dds/merge-tree/src/snapshotLoader.ts:24-253) for
// BatchClients: many documents' snapshots loaded into one BatchEngine at once.
//
//   const { loadSnapshots } = require("./snapshotLoader.js");
//   const catchup = loadSnapshots(engine, [{ client, snapshot }, ...]);  // then client.applyMsg(...)
//
// A snapshot is an ITree ({entries: [...]}, a SharedString keeps the merge-tree under "content";
// e.g. sequence/src/test/snapshots/*.json) or the {path: chunk} form SnapshotV1.emit /
// mt_get_snapshot produce.  Chunks are brought to the v1 shape as toLatestVersion does
// (snapshotChunks.ts:133-185).  Then, as fluidframework_amd/snapshot.py on the Python side:
//   * the header's segments become the document through mt_docs_load (reloadFromSegments,
//     mergeTree.ts:1195-1251, + startOrUpdateCollaboration(minSeq, seq)) on the device;
//   * every body segment becomes an MT_OP_LOAD record applied by the engine's insert path as
//     loadBody's insertSegments(root.cachedLength, ...) (snapshotLoader.ts:192-224);
//   * catch-up ops (legacy) are returned per document, to be applied with applyMsg.
// specToSegment (snapshotLoader.ts:85-117): without merge info a segment is (seq 0, NonCollabClient).
const native = require("./mtgpu.node");

const MT_OP_LOAD = 4, F_PROPS = 2, F_MARKER = 128, OP_WIDE = 0x80;  // (npairs: BatchClient's encoder)
const NONCOLLAB = 0xfe, UNIVERSAL_SEQ = 0, SF_PDEF = 2, SF_MARKER = 16, LSF_U16 = 64, LOAD_SEG = 96;

function blobs(tree) {
    if (tree && Array.isArray(tree.entries)) {
        let entries = tree.entries;
        const content = entries.find((e) => e.path === "content" && e.type === "Tree");
        if (content) entries = content.value.entries;
        const out = {};
        for (const e of entries) if (e.type === "Blob") out[e.path] = e.value.contents;
        return out;
    }
    return Object.assign({}, tree);
}

const parse = (x) => (typeof x === "string" ? JSON.parse(x) : x);

function toLatestVersion(path, chunk) {  // snapshotChunks.ts:133-185
    if (chunk.version === "1") return chunk;
    if (chunk.version !== undefined) throw new Error(`Unsupported chunk path: ${path} version: ${chunk.version}`);
    let meta;
    if (path === "header") {
        meta = chunk.headerMetadata;
        if (meta === undefined) {
            const ids = [{ id: "header" }];
            if (chunk.chunkLengthChars < chunk.totalLengthChars) ids.push({ id: "body" });
            meta = { orderedChunkMetadata: ids, minSequenceNumber: chunk.chunkMinSequenceNumber,
                sequenceNumber: chunk.chunkSequenceNumber, totalLength: chunk.totalLengthChars,
                totalSegmentCount: chunk.totalSegmentCount };
        }
    }
    return { version: "1", length: chunk.chunkLengthChars, segmentCount: chunk.chunkSegmentCount,
        headerMetadata: meta, segments: chunk.segmentTexts, startIndex: chunk.chunkStartSegmentIndex };
}

function parseDoc(tree) {
    const b = blobs(tree);
    const header = toLatestVersion("header", parse(b.header));
    const meta = header.headerMetadata;
    if (!meta) throw new Error("header metadata not available");
    const body = [];
    if (header.segmentCount !== meta.totalSegmentCount) {  // snapshotLoader.ts:159-190
        for (const md of meta.orderedChunkMetadata.slice(1)) body.push(...toLatestVersion(md.id, parse(b[md.id])).segments);
    }
    const known = new Set(meta.orderedChunkMetadata.map((m) => m.id));
    const rest = Object.keys(b).filter((p) => !known.has(p));
    if (rest.length > 1) throw new Error("Unexpected blobs in snapshot");
    const catchup = rest.length === 1 && b[rest[0]] ? parse(b[rest[0]]) : [];
    const seq = meta.sequenceNumber;
    const minSeq = meta.minSequenceNumber !== undefined && meta.minSequenceNumber !== null ? meta.minSequenceNumber : seq;
    return { header: header.segments, body, catchup, seq, minSeq };
}

// specToSegment -> {bytes, seq, client, rseq, rclient, pdef, pairs, marker}; ids interned by the client
function spec(client, s) {
    const merge = s !== null && typeof s === "object" && "json" in s;
    const js = merge ? s.json : s;
    let text, props, marker = false;
    if (typeof js === "string") {
        text = js;
    } else if (js && typeof js === "object" && "text" in js) {
        text = js.text; props = js.props;
    } else if (js && typeof js === "object" && "marker" in js) {  // Marker.fromJSONObject (mergeTree.ts:658-665)
        const rt = js.marker.refType || 0;
        if (!(Number.isInteger(rt) && rt >= 0 && rt <= 255)) throw new Error("snapshotLoader: marker refType out of range");
        text = String.fromCharCode(rt); props = js.props; marker = true;
    } else {
        throw new Error("snapshotLoader: not a text or marker segment spec");
    }
    // UTF-16 code units (cachedLength = text.length, textSegment.ts:45): Latin-1 bytes when they fit
    const u16 = /[^\u0000-\u00ff]/.test(text);
    let pairs = [];
    if (props !== undefined && props !== null) {
        const nonNull = {};
        for (const k of Object.keys(props)) if (props[k] !== null) nonNull[k] = props[k];
        pairs = client._pairs(nonNull);
    }
    let seq = UNIVERSAL_SEQ, c = NONCOLLAB, rseq = -1, rc = 0;
    if (merge) {
        if (s.seq !== undefined && s.seq !== null) seq = s.seq;
        if (s.client !== undefined && s.client !== null) c = client._shortId(s.client);
        if (s.removedSeq !== undefined && s.removedSeq !== null) rseq = s.removedSeq;
        if (s.removedClient !== undefined && s.removedClient !== null) rc = client._shortId(s.removedClient);
    }
    let wide = u16 || (c >= 64 && c !== NONCOLLAB) || (rseq >= 0 && rc >= 64);  // the wide form (include/mtgpu.h)
    for (let q = 0; q < pairs.length; q += 2) wide = wide || pairs[q] >= 8 || pairs[q + 1] > 255;
    return { bytes: Buffer.from(text, wide ? "utf16le" : "latin1"), units: text.length, u16: wide, seq, client: c,
        rseq, rclient: rc, pdef: props !== undefined && props !== null, pairs, marker, wide };
}

/**
 * Load one snapshot per BatchClient (entries: [{client, snapshot}], the clients of `engine`, whose
 * collaboration has started and which have applied nothing yet).  Returns the catch-up messages
 * of each entry, to be applied with client.applyMsg.
 */
function loadSnapshots(engine, entries) {
    engine.flush();
    const n = entries.length;
    const docIds = new Uint32Array(n), segRow = new Uint32Array(n + 1);
    const minSeq = new Int32Array(n), curSeq = new Int32Array(n);
    const segRows = [], texts = [];
    let nseg = 0, textOff = 0;
    const parsed = entries.map((e) => parseDoc(e.snapshot));
    entries.forEach(({ client }, i) => {
        if (client.engine !== engine) throw new Error("snapshotLoader: client of another engine");
        if (client.queue.length || client.currentSeq) throw new Error("snapshotLoader: the client has applied ops");
        const doc = parsed[i];
        docIds[i] = client.doc;
        let local = 0;  // root.cachedLength: the local (non-removed) length
        for (const s of doc.header) {
            const x = spec(client, s);
            const row = Buffer.alloc(LOAD_SEG);  // mt_load_seg (include/mtgpu.h)
            row.writeInt32LE(x.seq, 0); row.writeInt32LE(x.rseq, 4);
            const rc = x.rseq >= 0 ? x.rclient : 0;
            row.writeUInt8(x.client & 0xff, 8); row.writeUInt8(rc & 0xff, 9);
            row.writeUInt8(x.client >> 8, 20); row.writeUInt8(rc >> 8, 21);  // client_hi, rclient_hi
            row.writeUInt8((x.pdef ? SF_PDEF : 0) | (x.marker ? SF_MARKER : 0) | (x.u16 ? LSF_U16 : 0), 10);
            row.writeUInt32LE(textOff, 12); row.writeUInt32LE(x.units, 16);
            for (let q = 0; q < x.pairs.length; q += 2) row.writeUInt16LE(x.pairs[q + 1], 24 + 2 * x.pairs[q]);
            segRows.push(row); texts.push(x.bytes);
            textOff += x.bytes.length; nseg++;
            if (x.rseq < 0) local += x.units;
        }
        segRow[i + 1] = nseg;
        minSeq[i] = doc.minSeq; curSeq[i] = doc.seq;
        // loadBody (snapshotLoader.ts:192-224): a run of specs without merge info is one
        // insertSegments at root.cachedLength, each next one at insertPos += cachedLength
        let batchPos = null;
        for (const s of doc.body) {
            const x = spec(client, s);
            const batched = x.client === NONCOLLAB && x.seq === UNIVERSAL_SEQ;
            let pos;
            if (batched) {
                pos = batchPos === null ? local : batchPos;
                batchPos = pos + x.units;
            } else {
                pos = local;
                batchPos = null;
            }
            if (x.rseq < 0) local += x.units;
            const sorted = [];
            for (let q = 0; q < x.pairs.length; q += 2) sorted.push([x.pairs[q], x.pairs[q + 1]]);
            sorted.sort((a, b) => a[0] - b[0]);
            const pb = Buffer.alloc((x.wide ? 3 : 2) * sorted.length);
            sorted.forEach(([k, v], q) => {
                if (x.wide) { pb.writeUInt8(k, 3 * q); pb.writeUInt16LE(v, 3 * q + 1); } else { pb.writeUInt8(k, 2 * q); pb.writeUInt8(v, 2 * q + 1); }
            });
            // (MT_OP_LOAD: the short ids' low bytes in `client`, their high bytes in `msn`)
            const rc = x.rseq >= 0 ? x.rclient : 0;
            client.queue.push({ seq: x.seq, ref: UNIVERSAL_SEQ, msn: (x.client >> 8) | ((rc >> 8) << 8),
                client: (x.client & 0xff) | ((rc & 0xff) << 8), type: MT_OP_LOAD | (x.wide ? OP_WIDE : 0),
                flags: (x.pdef ? F_PROPS : 0) | (x.marker ? F_MARKER : 0), npairs: sorted.length, pos1: pos,
                pos2: x.rseq, payload: Buffer.concat([x.bytes, pb]) });
            engine.pending++;
        }
        client.currentSeq = doc.seq;
        client.minSeq = doc.minSeq;
    });
    engine.gen++;  // (segment descriptors of the loaded documents are stale from here on)
    native.docsLoad(engine.handle, docIds, segRow, Buffer.concat(segRows.length ? segRows : [Buffer.alloc(0)]),
        Buffer.concat(texts.length ? texts : [Buffer.alloc(0)]), minSeq, curSeq);
    engine.flush();  // the body appends
    return parsed.map((d) => d.catchup);
}

module.exports = { loadSnapshots, parseDoc, toLatestVersion };
