"use strict";
// An editing client through the Node surface: each document of a local_* log (tests/golden/
// make_local.py) replayed into a BatchClient "c<own>" -- its local edits through insertTextLocal /
// removeRangeLocal / annotateRangeLocal, the sequenced stream (its own messages = acks) through
// applyMsg -- one JSON line per document {doc, err, state}.
//   node replay_local.js <log.mtlog>
const { BatchEngine } = require("./batchClient.js");
const { loadLog, messages } = require("./mtlog.js");

// an op as [type, pos1, pos2, text | null, {key id: value | null} | null, flags] (replay_ref.js opTuple)
function tuple(op) {
    const props = (p) => {
        if (!p) return null;
        const o = {};
        for (const k of Object.keys(p)) o[parseInt(k.slice(1), 10)] = p[k];
        return o;
    };
    if (op.type === 0) {
        const seg = op.seg;
        if (seg.marker) return [0, op.pos1, 0, String.fromCharCode(seg.marker.refType), props(seg.props), 128];
        return [0, op.pos1, 0, typeof seg === "string" ? seg : seg.text, typeof seg === "string" ? null : props(seg.props), 0];
    }
    if (op.type === 1) return [1, op.pos1, op.pos2, null, null, 0];
    return [2, op.pos1, op.pos2, null, props(op.props), op.combiningOp && op.combiningOp.name === "rewrite" ? 1 : 0];
}

const log = loadLog(process.argv[2]);
const withEvents = process.argv[3] === "events";
// "seqdelta": SequenceDeltaEvents (js/sequenceDeltaEvent.js) from a "sequenceDelta" listener, one record
// per event in replay_ref.js's seqdelta form
const withSeqDelta = process.argv[3] === "seqdelta";
// "read": the read surface over each document's final state, in replay_ref.js's read form
const withRead = process.argv[3] === "read";
// "seqreads": what a listener reads inside each delta callback (getText, getLength, getPosition of the
// delta segments), callbacks delivered synchronously (BatchEngine syncCallbacks), in replay_ref.js's
// seqreads form; argv[4]: the first documents only
const withReads = process.argv[3] === "seqreads";
const nReads = withReads && process.argv[4] ? parseInt(process.argv[4], 10) : Infinity;
const { SequenceEvents } = require("./sequenceDeltaEvent.js");
const eng = new BatchEngine({ maxDocs: log.nDocs, opsPerLaunch: 16, syncCallbacks: withReads });
const sortKeys = (pd) => {
    const o = {};
    for (const k of Object.keys(pd).sort((a, b) => parseInt(a.slice(1), 10) - parseInt(b.slice(1), 10))) o[k] = pd[k];
    return o;
};
const clients = [];
for (let d = 0; d < log.nDocs; d++) {
    const items = [...messages(log, d)];
    const own = items.find((x) => x.local);
    const c = eng.createClient();
    c.startOrUpdateCollaboration(own ? "c" + own.client : "observer");
    const regen = [];
    c.events = [];
    if (withEvents) {  // the canonical event form of fluidframework_amd/events.py; a local edit's seq is -1
        const seg = (x, pd) => [x.segment.ordinal, x.segment.position === undefined ? -1 : x.segment.position,
            x.segment.cachedLength, pd];
        c.mergeTreeDeltaCallback = (opArgs, args) => c.events.push([
            opArgs.sequencedMessage ? opArgs.sequencedMessage.sequenceNumber : -1, args.operation,
            args.deltaSegments.map((x) => seg(x, args.operation === 2 && x.propertyDeltas ? sortKeys(x.propertyDeltas) : null))]);
        c.mergeTreeMaintenanceCallback = (args) => c.events.push([args.sequenceNumber, args.operation,
            args.deltaSegments.map((x) => seg(x, null))]);
    }
    if (withReads && d < nReads) {
        c.mergeTreeDeltaCallback = (opArgs, args) => c.events.push([
            opArgs.sequencedMessage ? opArgs.sequencedMessage.sequenceNumber : -1, c.getText(), c.getLength(),
            args.deltaSegments.map((x) => c.getPosition(x.segment))]);
    }
    if (withSeqDelta) {
        const seqEvents = new SequenceEvents(c);
        seqEvents.on("sequenceDelta", (ev) => {
            const ranges = ev.ranges.map((r) => [r.operation, r.segment.ordinal, r.position, r.segment.cachedLength,
                r.propertyDeltas ? sortKeys(r.propertyDeltas) : null]);
            const m = ev.opArgs.sequencedMessage;
            c.events.push([m ? m.sequenceNumber : -1, ev.deltaOperation, ev.isLocal, ev.isEmpty, ev.clientId, ranges,
                ev.first ? ev.first.segment.ordinal : null, ev.last ? ev.last.segment.ordinal : null]);
        });
    }
    c.remoteIds = new Set();
    for (const it of items) {
        if (!it.local && !it.regen) c.remoteIds.add(it.clientId);
        if (it.regen) {  // reconnect: the op to resubmit, as record tuples
            const op = c.regeneratePendingOp(it.op);
            regen.push([it.index, (op.type === 3 ? op.ops : [op]).map(tuple)]);
            continue;
        }
        if (!it.local) {
            c.applyMsg(it);
            continue;
        }
        const op = it.op;
        let r;
        if (op.type === 0) {
            r = typeof op.seg === "string" ? c.insertTextLocal(op.pos1, op.seg)
                : op.seg.marker ? c.insertMarkerLocal(op.pos1, op.seg.marker.refType, op.seg.props)
                    : c.insertTextLocal(op.pos1, op.seg.text, op.seg.props);
        } else if (op.type === 1) {
            r = c.removeRangeLocal(op.pos1, op.pos2);
        } else {
            r = c.annotateRangeLocal(op.pos1, op.pos2, op.props, op.combiningOp);
        }
        if (!r) throw new Error("local edit rejected");
    }
    c.regen = regen;
    clients.push(c);
}
function readSurface(c, d) {
    const pset = (seg) => (seg && seg.properties ? sortKeys(seg.properties) : null);
    const len = c.getLength();
    const positions = [];
    const stride = Math.max(1, Math.floor((len + 2) / 48));
    for (let p = 0; p <= len + 1; p += stride) positions.push(p);
    if (positions[positions.length - 1] !== len) positions.push(len);
    const contain = positions.map((p) => {
        const r = c.getContainingSegment(p);
        return r.segment ? [r.segment.ordinal, r.offset] : null;
    });
    const props = positions.map((p) => pset(c.getContainingSegment(p).segment));
    const extents = positions.map((p) => {
        const e = c.getRangeExtentsOfPosition(p);
        return [e.posStart === undefined ? null : e.posStart, e.posAfterEnd === undefined ? null : e.posAfterEnd];
    });
    const walks = [];
    for (const [a, b, stop] of [[undefined, undefined, 0], [Math.floor(len / 3), Math.floor((2 * len) / 3) + 1, 0],
        [1, len, 3], [len, len + 5, 0]]) {
        const calls = [];
        c.walkSegments((seg, pos, refSeq, clientId, start, end) => {
            calls.push([seg.ordinal, pos, start, end]);
            return stop === 0 || calls.length < stop;
        }, a, b);
        walks.push(calls);
    }
    const getpos = c._segments().map((seg) => c.getPosition(seg));
    const remote = [];
    const seq = c.getCurrentSeq();
    for (const id of [...c.remoteIds].sort().slice(0, 4)) {
        for (const refSeq of (c.longClientId !== "observer") ? [seq] : [Math.max(c.getState().msn, seq - 5), seq]) {
            const cid = c._shortId(id);
            const local = cid === c._shortId(c.longClientId);
            const rl = c._segments().reduce((acc, x) => acc + c.constructor._viewLength(x, refSeq, cid, local), 0);
            for (const p of [0, Math.floor(rl / 2), rl, rl + 1]) {
                const r = c.resolveRemoteClientPosition(p, refSeq, id);
                remote.push([id, refSeq, p, r === undefined ? null : r]);
            }
        }
    }
    return { doc: d, err: null, len, positions, contain, props, extents, walks, getpos, remote };
}
const out = clients.map((c, d) => {
    if (withRead) {
        try { return JSON.stringify(readSurface(c, d)); } catch (e) { return JSON.stringify({ doc: d, err: String(e.message || e) }); }
    }
    let err = null, state = null;
    try { state = c.getState(); } catch (e) { err = String(e.message || e); }
    const line = c.regen.length ? { doc: d, err, state, regen: c.regen } : { doc: d, err, state };
    if (withEvents || withSeqDelta) line.events = c.events;
    if (withReads) return JSON.stringify({ doc: d, err, reads: c.events });
    return JSON.stringify(line);
});
process.stdout.write(out.join("\n") + "\n");
