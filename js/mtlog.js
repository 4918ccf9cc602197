"use strict";
// mtlog.js -- read MTLOG op-log files (fluidframework_amd/oplog.py) as ISequencedDocumentMessage
// objects (protocol.ts:132-172) carrying IMergeTreeOp contents (ops.ts:63-110).  Client long ids
// are "c<id>" for record client <id>; property keys "k<id>", values the value ids.  A marker insert
// (flags bit 7) carries its ReferenceType as the one text byte: seg = {marker: {refType}, props?}.
const fs = require("fs");

function loadLog(file) {
    const buf = fs.readFileSync(file);
    if (buf.toString("latin1", 0, 8) !== "MTLOG001") throw new Error("not an MTLOG file");
    const nDocs = buf.readUInt32LE(8);
    const nOps = Number(buf.readBigUInt64LE(16));
    let off = 32;
    const rowPtr = new Uint32Array(nDocs + 1);
    for (let i = 0; i <= nDocs; i++) rowPtr[i] = buf.readUInt32LE(off + 4 * i);
    off += 4 * (nDocs + 1);
    return { buf, nDocs, nOps, rowPtr, opsOff: off, payOff: off + 32 * nOps };
}

function readOp(log, i) {
    const b = log.buf, o = log.opsOff + 32 * i;
    return {
        seq: b.readInt32LE(o), ref: b.readInt32LE(o + 4), msn: b.readInt32LE(o + 8),
        client: b.readUInt16LE(o + 12), type: b.readUInt8(o + 14), flags: b.readUInt8(o + 15),
        pos1: b.readInt32LE(o + 16), pos2: b.readInt32LE(o + 20),
        poff: b.readUInt32LE(o + 24), plen: b.readUInt32LE(o + 28),
    };
}

// Tile-label logs (opts.tileKey = k): key k is the reserved "referenceTileLabels" property
// (mergeTree.ts:575) and its value id v the label array ["L<i>" for every bit i of v]; the same
// for opts.rangeKey and "referenceRangeLabels" (mergeTree.ts:576)
function tileLabels(v) {
    const out = [];
    for (let i = 0; i < 8; i++) if ((v >> i) & 1) out.push("L" + i);
    return out;
}

// a record's payload: [text][pairs]; narrow: Latin-1 bytes and (key u8, value u8) pairs; wide
// (type bit 7, MT_OP_WIDE): UTF-16 LE code units and (key u8, value u16 LE) pairs
const pairBytes = (r) => (r.type & 0x80 ? 3 : 2);
// property pairs: flags bits 3..6, plus 16 when type bit 6 (MT_OP_NP16) is set, 32 when type bit 5
// (MT_OP_NP32) is
const npairsOf = (r) => ((r.flags >> 3) & 15) | (r.type & 0x40 ? 16 : 0) | (r.type & 0x20 ? 32 : 0);
function textOf(log, r) {
    const np = npairsOf(r);
    const a = log.payOff + r.poff, b = a + r.plen - pairBytes(r) * np;
    return log.buf.toString(r.type & 0x80 ? "utf16le" : "latin1", a, b);
}

function propsOf(log, r, opts) {
    const np = npairsOf(r), pb = pairBytes(r);
    const start = log.payOff + r.poff + r.plen - pb * np;
    const props = {};
    for (let q = 0; q < np; q++) {
        const k = log.buf.readUInt8(start + pb * q);
        const v = pb === 3 ? log.buf.readUInt16LE(start + 3 * q + 1) : log.buf.readUInt8(start + 2 * q + 1);
        if (opts && opts.tileKey === k) props.referenceTileLabels = v === 0 ? null : tileLabels(v);
        else if (opts && opts.rangeKey === k) props.referenceRangeLabels = v === 0 ? null : tileLabels(v);
        else props["k" + k] = v === 0 ? null : v;
    }
    return props;
}

function toOp(log, r, opts) {
    const type = r.type & 0x1f;
    if (type === 0 && (r.flags & 128)) {
        const seg = { marker: { refType: textOf(log, r).charCodeAt(0) } };
        if (r.flags & 2) seg.props = propsOf(log, r, opts);
        return { type: 0, pos1: r.pos1, seg };
    }
    if (type === 0) {
        const text = textOf(log, r);
        return { type: 0, pos1: r.pos1, seg: (r.flags & 2) ? { text, props: propsOf(log, r, opts) } : text };
    }
    if (type === 1) return { type: 1, pos1: r.pos1, pos2: r.pos2 };
    if (type === 2) {
        const op = { type: 2, pos1: r.pos1, pos2: r.pos2, props: propsOf(log, r, opts) };
        if (r.flags & 1) op.combiningOp = { name: "rewrite" };
        return op;
    }
    return undefined;
}

function msgOf(r, op) {
    return {
        clientId: "c" + r.client, clientSequenceNumber: 1, contents: op, metadata: undefined,
        minimumSequenceNumber: r.msn, origin: undefined, referenceSequenceNumber: r.ref,
        sequenceNumber: r.seq, timestamp: 0, term: 1, traces: [], type: op ? "op" : "noop",
    };
}

/** The messages of document d, GROUP members folded into one message (client.ts:782-790); a record
 * with seq -1 is a local edit of the document's editing client: {local: true, client, op, index}. */
function* messages(log, d, opts) {
    let group = null;
    for (let i = log.rowPtr[d]; i < log.rowPtr[d + 1]; i++) {
        const r = readOp(log, i);
        const op = toOp(log, r, opts);
        if (group || (r.flags & 4)) {
            if (!group) group = { r, ops: [] };
            if (op) group.ops.push(op);
            if (r.flags & 4) continue;
            const g = group;
            group = null;
            const m = msgOf(g.r, { type: 3, ops: g.ops });
            Object.defineProperty(m, "end", { value: i + 1 - log.rowPtr[d] });  // records consumed so far
            yield m;
            continue;
        }
        if (r.seq === -1) {  // an edit of the document's local client (seq UnassignedSequenceNumber)
            yield { local: true, client: r.client, op, index: i - log.rowPtr[d], end: i + 1 - log.rowPtr[d] };
            continue;
        }
        if (r.seq === -2) {  // reconnect: the local client regenerates this pending op (regeneratePendingOp)
            yield { regen: true, client: r.client, op, index: i - log.rowPtr[d], end: i + 1 - log.rowPtr[d] };
            continue;
        }
        const m = msgOf(r, op);
        Object.defineProperty(m, "end", { value: i + 1 - log.rowPtr[d] });
        yield m;
    }
}

module.exports = { loadLog, messages, tileLabels };
