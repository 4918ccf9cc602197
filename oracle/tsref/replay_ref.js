"use strict";
// Replays an MTLOG op log through the REFERENCE merge-tree (type-stripped into oracle/_tsref by
// build_ref.py) with one observer Client per document -- exactly the reference's own observer
// pattern (clientReplayTool.ts:193-255; mergeTreeOperationRunner.ts:163-178 client 0) -- and
// prints one canonical-state JSON line per document (DESIGN.md "Canonical state").
// TEST INFRASTRUCTURE ONLY (this container; the reference never travels to the GPU box).
//
//   node replay_ref.js state <log.mtlog> [d0 d1]     -> JSON lines {doc, err, state}
//   node replay_ref.js errstate <log.mtlog>           -> JSON lines {doc, err, err_msg_index, err_seq,
//        state}: where applyMsg throws, the thrown message, the index and sequenceNumber of the
//        message that threw, and the state after the messages BEFORE it (the reference leaves a
//        half-applied op behind a throw; the engine halts the document before the failing op)
//   node replay_ref.js bench <log.mtlog> <threads>   -> ops/sec over all docs (worker_threads)
//   node replay_ref.js snapshot <log.mtlog> [d0 d1 [chunk]]  -> JSON lines {doc, err, snapshot}: the
//        entries SnapshotV1.extractSync() + emit() write (snapshotV1.ts:85-246), path -> contents
//   node replay_ref.js load <log.mtlog> <k> [chunk]  -> JSON lines {doc, err, snapshot, state}: messages
//        [0, k) replayed on an observer, its SnapshotV1 tree loaded into a fresh Client through the
//        reference's SnapshotLoader (snapshotLoader.ts:35-225, MockStorage), then messages [k, n)
//        applied to the loaded Client; state = its canonical state
//   node replay_ref.js loadtree <snapshot.json> [log.mtlog]  -> one JSON line {err, state}: a stored
//        SharedString snapshot tree (its "content" subtree, e.g. sequence/src/test/snapshots/*) loaded
//        the same way, then the log's document 0 applied
const fs = require("fs");
const path = require("path");
const { Worker, isMainThread, parentPort, workerData } = require("worker_threads");

const ROOT = path.join(__dirname, "..", "_tsref", "merge-tree", "src");
const { Client } = require(path.join(ROOT, "client.js"));
const { TextSegment } = require(path.join(ROOT, "textSegment.js"));
const { MergeTree, Marker } = require(path.join(ROOT, "mergeTree.js"));
const { SnapshotV1 } = require(path.join(ROOT, "snapshotV1.js"));
const { SnapshotLoader } = require(path.join(ROOT, "snapshotLoader.js"));
const { MockStorage } = require(path.join(__dirname, "..", "_tsref", "node_modules", "@fluidframework",
    "test-runtime-utils", "mockStorage.js"));

const { loadLog, messages } = require(path.join(__dirname, "..", "..", "js", "mtlog.js"));

// the segment factory a SharedString uses (sequence/src/sharedString.ts segmentFromSpec): text or marker
function specToSegment(spec) { return TextSegment.fromJSONObject(spec) || Marker.fromJSONObject(spec); }

// a merge-tree op as an op-record tuple [type, pos1, pos2, text | null, {key id: value id | null} | null,
// flags] (F_REWRITE 1, F_MARKER 128; local_farm.js writes the same form)
function opTuple(op) {
    const props = (p) => {
        if (!p) return null;
        const o = {};
        for (const k of Object.keys(p)) o[parseInt(k.slice(1), 10)] = p[k] === undefined ? null : p[k];
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

function newObserver() {
    const logger = { send() {}, sendTelemetryEvent() {}, sendErrorEvent() {}, sendPerformanceEvent() {} };
    const c = new Client(specToSegment, logger);
    c.startOrUpdateCollaboration("observer");
    return c;
}

function logId(client, shortId) {
    if (shortId < 0) return -2;  // NonCollabClient (constants.ts:15): segments loaded below the MSN
    const long = client.getLongClientId(shortId);
    return long === "observer" ? 0 : parseInt(long.slice(1), 10);
}

function canonical(client) {
    const mt = client.mergeTree;
    const segs = [];
    const walk = (b) => {
        for (let i = 0; i < b.childCount; i++) {
            const ch = b.children[i];
            if (!ch.isLeaf()) { walk(ch); continue; }
            const removed = ch.removedSeq !== undefined;
            const ov = (ch.removedClientOverlap || []).map((x) => logId(client, x)).sort((a, b) => a - b);
            let props = null;
            if (ch.properties) {
                props = {};
                for (const k of Object.keys(ch.properties).sort((a, b) => parseInt(a.slice(1)) - parseInt(b.slice(1)))) {
                    props[k] = ch.properties[k];
                }
            }
            segs.push([Marker.is(ch) ? { marker: ch.refType } : ch.text, ch.seq, logId(client, ch.clientId), removed ? ch.removedSeq : -1,
                removed ? logId(client, ch.removedClientId) : -1, ov, props]);
        }
    };
    walk(mt.root);
    const tree = [];
    let lvl = [mt.root];
    while (lvl.length) {
        tree.push(lvl.map((b) => b.childCount));
        const nxt = [];
        for (const b of lvl) for (let i = 0; i < b.childCount; i++) if (!b.children[i].isLeaf()) nxt.push(b.children[i]);
        lvl = nxt;
    }
    const w = mt.getCollabWindow();
    return { seq: w.currentSeq, msn: w.minSeq, segs, tree };
}

// Delta / maintenance callbacks of an observer (mergeTreeDeltaCallback.ts:15-73; fired at
// mergeTree.ts:1981-1988, 2231-2236, 1310-1315, 1335-1340, 2592-2600, 2705-2712) in the canonical
// event form (DESIGN.md "Delta events"): [seq, operation, [[leaf, pos, len, propertyDeltas], ...]]
//   leaf = the segment's ordinal among the leaves still linked (segment.parent !== undefined) at
//          callback time, in document order; -1 when it is not linked (a zero-length insert);
//          a SPLIT's second segment is not linked yet: the first one's ordinal + 1
//   pos  = op callbacks: the local-view position (sum of localNetLength of the linked leaves
//          before it); maintenance callbacks: -1
//   len  = segment.cachedLength at callback time
//   propertyDeltas = ANNOTATE: {k<id>: previous value id | null} with sorted keys, else null
function attachEvents(c, seqRef) {
    const events = [];
    const where = (seg) => {
        let ord = 0, pos = 0, found = null;
        const walk = (b) => {
            for (let i = 0; i < b.childCount && !found; i++) {
                const ch = b.children[i];
                if (!ch.isLeaf()) { walk(ch); continue; }
                if (ch.parent === undefined) continue;
                if (ch === seg) { found = [ord, pos]; return; }
                ord++;
                pos += ch.removedSeq === undefined ? ch.cachedLength : 0;
            }
        };
        walk(c.mergeTree.root);
        return found || [-1, -1];
    };
    const pdelta = (pd) => {
        if (!pd) return null;
        const o = {};
        for (const k of Object.keys(pd).sort((a, b) => parseInt(a.slice(1)) - parseInt(b.slice(1)))) {
            o[k] = pd[k] === undefined ? null : pd[k];
        }
        return o;
    };
    c.mergeTreeDeltaCallback = (opArgs, args) => {
        const segs = args.deltaSegments.map((d) => {
            const [leaf, pos] = where(d.segment);
            return [leaf, pos, d.segment.cachedLength, args.operation === 2 ? pdelta(d.propertyDeltas) : null];
        });
        events.push([seqRef.seq, args.operation, segs]);
    };
    c.mergeTreeMaintenanceCallback = (args) => {
        const segs = [];
        for (let i = 0; i < args.deltaSegments.length; i++) {
            const seg = args.deltaSegments[i].segment;
            let leaf = where(seg)[0];
            if (args.operation === -2 && i === 1) leaf = segs[0][0] + 1;  // SPLIT: `next` not yet linked
            segs.push([leaf, -1, seg.cachedLength, null]);
        }
        events.push([seqRef.seq, args.operation, segs]);
    };
    return events;
}

function replayDoc(log, d) {
    const items = [...messages(log, d)];
    const own = items.find((x) => x.local);
    let c;
    if (own) {  // an editing client's log (seq -1 local edits, seq -2 reconnects; "local" mode)
        const logger = { send() {}, sendTelemetryEvent() {}, sendErrorEvent() {}, sendPerformanceEvent() {} };
        c = new Client(specToSegment, logger);
        c.startOrUpdateCollaboration("c" + own.client);
    } else {
        c = newObserver();
    }
    let err = null;
    try {
        for (const it of items) {
            if (it.regen) {
                c.regeneratePendingOp(it.op, c.mergeTree.pendingSegments.first());
            } else if (it.local) {
                const op = it.op;
                if (op.type === 0) c.insertSegmentLocal(op.pos1, specToSegment(op.seg));
                else if (op.type === 1) c.removeRangeLocal(op.pos1, op.pos2);
                else c.annotateRangeLocal(op.pos1, op.pos2, op.props, op.combiningOp);
            } else {
                c.applyMsg(it);
            }
        }
    } catch (e) {
        err = String(e.message || e);
    }
    return { c, err };
}

// SharedSegmentSequence.loadCore's view of the merge-tree content (a fresh Client, SnapshotLoader
// .initialize over the "content" blobs, then the catch-up ops), with the runtime pieces the loader
// reads stubbed: options, documentId, clientId (-> "snapshot", snapshotLoader.ts:145), attached.
async function loadClient(tree) {
    const logger = { send() {}, sendTelemetryEvent() {}, sendErrorEvent() {}, sendPerformanceEvent() {},
        shipAssert(c, e) { if (!c) throw new Error(`shipAssert ${JSON.stringify(e)}`); } };
    const c = new Client(specToSegment, logger);
    const runtime = { options: {}, documentId: "doc", clientId: undefined, attachState: "Attached", logger,
        IFluidSerializer: undefined };
    const loader = new SnapshotLoader(runtime, c, c.mergeTree, logger);
    const { catchupOpsP } = await loader.initialize("doc", new MockStorage(tree));
    const catchup = await catchupOpsP;
    for (const m of catchup) c.applyMsg(m);
    return c;
}

function emitTree(c, chunk) {
    const logger = { send() {}, sendTelemetryEvent() {}, sendErrorEvent() {}, sendPerformanceEvent() {} };
    if (chunk) {
        c.mergeTree.options = Object.assign({}, c.mergeTree.options, { mergeTreeSnapshotChunkSize: chunk });
    }
    const snap = new SnapshotV1(c.mergeTree, logger);
    snap.extractSync();
    return snap.emit();
}

async function mainAsync(mode) {
    if (mode === "load") {
        const log = loadLog(process.argv[3]);
        const k = parseInt(process.argv[4], 10);
        const chunk = process.argv[5] ? parseInt(process.argv[5], 10) : 0;
        const out = [];
        for (let d = 0; d < log.nDocs; d++) {
            const msgs = Array.from(messages(log, d));
            const c0 = newObserver();
            let err = null, snapshot = null, state = null;
            try {
                for (let i = 0; i < Math.min(k, msgs.length); i++) c0.applyMsg(msgs[i]);
                const tree = emitTree(c0, chunk);
                snapshot = {};
                for (const e of tree.entries) snapshot[e.path] = JSON.parse(e.value.contents);
                let c = await loadClient(tree), at = -1;
                for (let i = k; i < msgs.length && at < 0; i++) {
                    try {
                        c.applyMsg(msgs[i]);
                    } catch (e) {
                        err = String(e.message || e);
                        at = i;
                    }
                }
                if (at >= 0) {  // the state before the failing message (the engine halts there)
                    c = await loadClient(tree);
                    for (let i = k; i < at; i++) c.applyMsg(msgs[i]);
                }
                state = canonical(c);
            } catch (e) {
                err = String(e.message || e);
            }
            out.push(JSON.stringify({ doc: d, err, snapshot, state }));  // (err: the message [k, n) that threw)
        }
        process.stdout.write(out.join("\n") + "\n");
        return;
    }
    if (mode === "loadtree") {
        const stored = JSON.parse(fs.readFileSync(process.argv[3], "utf8"));
        const content = stored.entries.find((e) => e.path === "content" && e.type === "Tree");
        const c = await loadClient(content ? content.value : stored);
        let err = null;
        if (process.argv[4]) {
            const log = loadLog(process.argv[4]);
            try {
                for (const m of messages(log, 0)) c.applyMsg(m);
            } catch (e) {
                err = String(e.message || e);
            }
        }
        process.stdout.write(JSON.stringify({ err, state: canonical(c) }) + "\n");
        return;
    }
    throw new Error("mode: state | errstate | snapshot | load | loadtree | bench");
}

function main() {
    if (process.argv[2] === "load" || process.argv[2] === "loadtree") {
        mainAsync(process.argv[2]).catch((e) => { console.error(e); process.exit(1); });
        return;
    }
    const mode = process.argv[2];
    const log = loadLog(process.argv[3]);
    if (mode === "state") {
        const d0 = process.argv[4] ? parseInt(process.argv[4], 10) : 0;
        const d1 = process.argv[5] ? parseInt(process.argv[5], 10) : log.nDocs;
        const out = [];
        for (let d = d0; d < d1; d++) {
            const { c, err } = replayDoc(log, d);
            out.push(JSON.stringify({ doc: d, err, state: canonical(c), text: c.createTextHelper().getText(c.getCurrentSeq(), c.getClientId()) }));
        }
        process.stdout.write(out.join("\n") + "\n");
        return;
    }
    if (mode === "events") {
        const d0 = process.argv[4] ? parseInt(process.argv[4], 10) : 0;
        const d1 = Math.min(log.nDocs, process.argv[5] ? parseInt(process.argv[5], 10) : log.nDocs);
        const out = [];
        for (let d = d0; d < d1; d++) {
            const c = newObserver(), seqRef = { seq: 0 };
            const events = attachEvents(c, seqRef);
            let err = null;
            try {
                for (const m of messages(log, d)) {
                    seqRef.seq = m.sequenceNumber;
                    c.applyMsg(m);
                }
            } catch (e) {
                err = String(e.message || e);
            }
            out.push(JSON.stringify({ doc: d, err, events }));
        }
        process.stdout.write(out.join("\n") + "\n");
        return;
    }
    if (mode === "tiles") {
        // findTile (client.ts:1073-1076, mergeTree.ts:1763-1789) on each document after its whole
        // log, key <tileKey> carrying the tile labels (mtlog.js tileLabels); queries: every label
        // L0..L3, both directions, at a spread of positions around and past the length
        const tileKey = parseInt(process.argv[4] || "7", 10);
        const out = [];
        for (let d = 0; d < log.nDocs; d++) {
            const c = newObserver();
            let err = null;
            try {
                for (const m of messages(log, d, { tileKey })) c.applyMsg(m);
            } catch (e) {
                err = String(e.message || e);
            }
            const len = c.getLength();
            const ps = Array.from(new Set([0, 1, 2, len >> 3, len >> 2, len >> 1, (3 * len) >> 2, len - 2, len - 1, len,
                len + 1].filter((p) => p >= 0))).sort((a, b) => a - b);
            const answers = [];
            for (const p of ps) {
                for (let l = 0; l < 4; l++) {
                    for (const preceding of [true, false]) {
                        const t = c.findTile(p, "L" + l, preceding);
                        answers.push([p, l, preceding ? 1 : 0, t ? t.pos : null]);
                    }
                }
            }
            out.push(JSON.stringify({ doc: d, err, len, answers }));
        }
        process.stdout.write(out.join("\n") + "\n");
        return;
    }
    if (mode === "local") {
        // an editing client (client.ts:163-214, 588-625): the document's records with seq -1 are its
        // local edits (insertSegmentLocal / removeRangeLocal / annotateRangeLocal), the rest the
        // sequenced stream it receives -- its own messages among them, acked.  States after
        // record counts k of a spread of checkpoints and at the end: [[k, state], ...]
        const nck = parseInt(process.argv[4] || "6", 10);
        const out = [];
        for (let d = 0; d < log.nDocs; d++) {
            const n = log.rowPtr[d + 1] - log.rowPtr[d];
            const items = [...messages(log, d)];
            const own = items.find((x) => x.local);
            const logger = { send() {}, sendTelemetryEvent() {}, sendErrorEvent() {}, sendPerformanceEvent() {} };
            const c = new Client(specToSegment, logger);
            c.startOrUpdateCollaboration(own ? "c" + own.client : "observer");
            const cks = new Set();
            for (let q = 1; q < nck; q++) cks.add(Math.floor((q * n) / nck));
            const states = [];
            const regen = [];
            let err = null, k = 0;
            try {
                for (const it of items) {
                    if (it.regen) {  // regeneratePendingOp of the oldest pending edit (client.ts:855-893)
                        const op2 = c.regeneratePendingOp(it.op, c.mergeTree.pendingSegments.first());
                        regen.push([it.index, (op2.type === 3 ? op2.ops : [op2]).map(opTuple)]);
                    } else if (it.local) {
                        const op = it.op;
                        let ok;
                        if (op.type === 0) ok = c.insertSegmentLocal(op.pos1, specToSegment(op.seg));
                        else if (op.type === 1) ok = c.removeRangeLocal(op.pos1, op.pos2);
                        else ok = c.annotateRangeLocal(op.pos1, op.pos2, op.props, op.combiningOp);
                        if (!ok) throw new Error("local edit rejected");
                    } else {
                        c.applyMsg(it);
                    }
                    k = it.end;  // records consumed (a GROUP message is several)
                    if (cks.has(k)) states.push([k, canonical(c)]);
                }
            } catch (e) {
                err = String(e.message || e);
            }
            states.push([k, canonical(c)]);
            out.push(JSON.stringify(regen.length ? { doc: d, err, states, regen } : { doc: d, err, states }));
        }
        process.stdout.write(out.join("\n") + "\n");
        return;
    }
    if (mode === "localevents") {
        // the delta / maintenance callbacks an editing client fires (local edits: seq -1; its
        // acks and remote ops: the message's seq), canonical form as in "events"
        const out = [];
        for (let d = 0; d < log.nDocs; d++) {
            const items = [...messages(log, d)];
            const own = items.find((x) => x.local);
            const logger = { send() {}, sendTelemetryEvent() {}, sendErrorEvent() {}, sendPerformanceEvent() {} };
            const c = new Client(specToSegment, logger);
            c.startOrUpdateCollaboration(own ? "c" + own.client : "observer");
            const seqRef = { seq: 0 };
            const events = attachEvents(c, seqRef);
            let err = null;
            try {
                for (const it of items) {
                    if (it.regen) {
                        seqRef.seq = -2;
                        c.regeneratePendingOp(it.op, c.mergeTree.pendingSegments.first());
                    } else if (it.local) {
                        seqRef.seq = -1;
                        const op = it.op;
                        if (op.type === 0) c.insertSegmentLocal(op.pos1, specToSegment(op.seg));
                        else if (op.type === 1) c.removeRangeLocal(op.pos1, op.pos2);
                        else c.annotateRangeLocal(op.pos1, op.pos2, op.props, op.combiningOp);
                    } else {
                        seqRef.seq = it.sequenceNumber;
                        c.applyMsg(it);
                    }
                }
            } catch (e) {
                err = String(e.message || e);
            }
            out.push(JSON.stringify({ doc: d, err, events }));
        }
        process.stdout.write(out.join("\n") + "\n");
        return;
    }
    if (mode === "seqdelta") {
        // SequenceDeltaEvent (packages/dds/sequence/src/sequenceDeltaEvent.ts, transpiled) around every
        // delta callback of the document's client (an editing client for a local_* log, else the
        // observer), its ranges read inside the listener as SharedString users do: one record per
        // event [seq (-1: local edit), deltaOperation, isLocal, isEmpty, clientId, [[operation, leaf,
        // position, cachedLength, propertyDeltas | null], ...], first leaf | null, last leaf | null]
        const { SequenceDeltaEvent } = require(path.join(__dirname, "..", "_tsref", "sequence", "src",
            "sequenceDeltaEvent.js"));
        const out = [];
        for (let d = 0; d < log.nDocs; d++) {
            const items = [...messages(log, d)];
            const own = items.find((x) => x.local);
            const logger = { send() {}, sendTelemetryEvent() {}, sendErrorEvent() {}, sendPerformanceEvent() {} };
            const c = new Client(specToSegment, logger);
            c.startOrUpdateCollaboration(own ? "c" + own.client : "observer");
            const seqRef = { seq: 0 };
            const leafOf = (seg) => {
                let ord = 0, found = -1;
                const walk = (b) => {
                    for (let i = 0; i < b.childCount && found < 0; i++) {
                        const ch = b.children[i];
                        if (!ch.isLeaf()) { walk(ch); continue; }
                        if (ch.parent === undefined) continue;
                        if (ch === seg) { found = ord; return; }
                        ord++;
                    }
                };
                walk(c.mergeTree.root);
                return found;
            };
            const pdelta = (pd) => {
                if (!pd) return null;
                const o = {};
                for (const k of Object.keys(pd).sort((a, b) => parseInt(a.slice(1)) - parseInt(b.slice(1)))) {
                    o[k] = pd[k] === undefined ? null : pd[k];
                }
                return o;
            };
            const events = [];
            c.mergeTreeDeltaCallback = (opArgs, deltaArgs) => {
                const ev = new SequenceDeltaEvent(opArgs, deltaArgs, c);
                const ranges = ev.ranges.map((r) => [r.operation, leafOf(r.segment), r.position, r.segment.cachedLength,
                    pdelta(r.propertyDeltas)]);
                events.push([seqRef.seq, ev.deltaOperation, ev.isLocal, ev.isEmpty, ev.clientId, ranges,
                    ev.first ? leafOf(ev.first.segment) : null, ev.last ? leafOf(ev.last.segment) : null]);
            };
            let err = null;
            try {
                for (const it of items) {
                    if (it.regen) {
                        seqRef.seq = -2;
                        c.regeneratePendingOp(it.op, c.mergeTree.pendingSegments.first());
                    } else if (it.local) {
                        seqRef.seq = -1;
                        const op = it.op;
                        if (op.type === 0) c.insertSegmentLocal(op.pos1, specToSegment(op.seg));
                        else if (op.type === 1) c.removeRangeLocal(op.pos1, op.pos2);
                        else c.annotateRangeLocal(op.pos1, op.pos2, op.props, op.combiningOp);
                    } else {
                        seqRef.seq = it.sequenceNumber;
                        c.applyMsg(it);
                    }
                }
            } catch (e) {
                err = String(e.message || e);
            }
            out.push(JSON.stringify({ doc: d, err, events }));
        }
        process.stdout.write(out.join("\n") + "\n");
        return;
    }
    if (mode === "seqreads") {
        // what a listener reads INSIDE each delta callback of the document's client (an editing client
        // for a local_* log, else the observer): SharedString.getText() (the client's view at its
        // collab window: textHelper.getText(currentSeq, clientId), sequence.ts), getLength(), and
        // getPosition(segment) of every delta segment -- one record per callback [seq (-1: local
        // edit), text, length, [position, ...]]
        const out = [];
        const d1 = Math.min(log.nDocs, process.argv[4] ? parseInt(process.argv[4], 10) : log.nDocs);
        for (let d = 0; d < d1; d++) {
            const items = [...messages(log, d)];
            const own = items.find((x) => x.local);
            const logger = { send() {}, sendTelemetryEvent() {}, sendErrorEvent() {}, sendPerformanceEvent() {} };
            const c = new Client(specToSegment, logger);
            c.startOrUpdateCollaboration(own ? "c" + own.client : "observer");
            const helper = c.createTextHelper();
            const seqRef = { seq: 0 };
            const reads = [];
            c.mergeTreeDeltaCallback = (opArgs, deltaArgs) => {
                const w = c.getCollabWindow();
                reads.push([seqRef.seq, helper.getText(w.currentSeq, w.clientId), c.getLength(),
                    deltaArgs.deltaSegments.map((s) => c.getPosition(s.segment))]);
            };
            let err = null;
            try {
                for (const it of items) {
                    if (it.regen) {
                        seqRef.seq = -2;
                        c.regeneratePendingOp(it.op, c.mergeTree.pendingSegments.first());
                    } else if (it.local) {
                        seqRef.seq = -1;
                        const op = it.op;
                        if (op.type === 0) c.insertSegmentLocal(op.pos1, specToSegment(op.seg));
                        else if (op.type === 1) c.removeRangeLocal(op.pos1, op.pos2);
                        else c.annotateRangeLocal(op.pos1, op.pos2, op.props, op.combiningOp);
                    } else {
                        seqRef.seq = it.sequenceNumber;
                        c.applyMsg(it);
                    }
                }
            } catch (e) {
                err = String(e.message || e);
            }
            out.push(JSON.stringify({ doc: d, err, reads }));
        }
        process.stdout.write(out.join("\n") + "\n");
        return;
    }
    if (mode === "read") {
        // the client's read surface over its final state (client.ts:275-311, 838-847, 1004-1040):
        // getContainingSegment / getPropertiesAtPosition / getRangeExtentsOfPosition at a spread of
        // positions, walkSegments over a few ranges, getPosition of every leaf and
        // resolveRemoteClientPosition for a few (pos, refSeq, client) -- segments as their leaf ordinal
        const out = [];
        for (let d = 0; d < log.nDocs; d++) {
            const items = [...messages(log, d)];
            const own = items.find((x) => x.local);
            const logger = { send() {}, sendTelemetryEvent() {}, sendErrorEvent() {}, sendPerformanceEvent() {} };
            const c = new Client(specToSegment, logger);
            c.startOrUpdateCollaboration(own ? "c" + own.client : "observer");
            let err = null;
            const clients = new Set();
            try {
                for (const it of items) {
                    if (it.regen) {
                        c.regeneratePendingOp(it.op, c.mergeTree.pendingSegments.first());
                    } else if (it.local) {
                        const op = it.op;
                        if (op.type === 0) c.insertSegmentLocal(op.pos1, specToSegment(op.seg));
                        else if (op.type === 1) c.removeRangeLocal(op.pos1, op.pos2);
                        else c.annotateRangeLocal(op.pos1, op.pos2, op.props, op.combiningOp);
                    } else {
                        c.applyMsg(it);
                        clients.add(it.clientId);
                    }
                }
            } catch (e) {
                err = String(e.message || e);
            }
            if (err) {
                out.push(JSON.stringify({ doc: d, err }));
                continue;
            }
            const leaves = [];
            const walk = (b) => {
                for (let i = 0; i < b.childCount; i++) {
                    const ch = b.children[i];
                    if (!ch.isLeaf()) walk(ch); else leaves.push(ch);
                }
            };
            walk(c.mergeTree.root);
            const ord = (seg) => leaves.indexOf(seg);
            const pset = (seg) => {
                if (!seg || !seg.properties) return null;
                const o = {};
                for (const k of Object.keys(seg.properties).sort((a, b) => parseInt(a.slice(1)) - parseInt(b.slice(1)))) {
                    o[k] = seg.properties[k] === undefined ? null : seg.properties[k];
                }
                return o;
            };
            const len = c.getLength();
            const positions = [];
            const stride = Math.max(1, Math.floor((len + 2) / 48));
            for (let p = 0; p <= len + 1; p += stride) positions.push(p);
            if (positions[positions.length - 1] !== len) positions.push(len);
            const contain = positions.map((p) => {
                const r = c.getContainingSegment(p);
                return r.segment ? [ord(r.segment), r.offset] : null;
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
                    calls.push([ord(seg), pos, start, end]);
                    return stop === 0 || calls.length < stop;
                }, a, b);
                walks.push(calls);
            }
            const getpos = leaves.map((seg) => c.getPosition(seg));
            const remote = [];
            const seq = c.getCurrentSeq();
            for (const id of [...clients].sort().slice(0, 4)) {
                for (const refSeq of (own) ? [seq] : [Math.max(c.getCollabWindow().minSeq, seq - 5), seq]) {
                    const rl = c.mergeTree.getLength(refSeq, c.getOrAddShortClientId(id));
                    for (const p of [0, Math.floor(rl / 2), rl, rl + 1]) {
                        const r = c.resolveRemoteClientPosition(p, refSeq, id);
                        remote.push([id, refSeq, p, r === undefined ? null : r]);
                    }
                }
            }
            out.push(JSON.stringify({ doc: d, err, len, positions, contain, props, extents, walks, getpos, remote }));
        }
        process.stdout.write(out.join("\n") + "\n");
        return;
    }
    if (mode === "stacks") {
        // getStackContext (client.ts:946-948, mergeTree.ts:1750-1760): the NestBegin / NestEnd stack of
        // each label L0..L3 at a spread of positions, range labels on key <rangeKey>; each stack as
        // [[marker position, refType], ...] bottom to top ([] when the label has none)
        const rangeKey = parseInt(process.argv[4] || "1", 10);
        const out = [];
        for (let d = 0; d < log.nDocs; d++) {
            const c = newObserver();
            let err = null;
            try {
                for (const m of messages(log, d, { rangeKey })) c.applyMsg(m);
            } catch (e) {
                err = String(e.message || e);
            }
            const len = c.getLength();
            const ps = Array.from(new Set([0, 1, 2, len >> 3, len >> 2, len >> 1, (3 * len) >> 2, len - 2, len - 1, len,
                len + 1].filter((p) => p >= 0))).sort((a, b) => a - b);
            const answers = [];
            for (const p of ps) {
                for (let l = 0; l < 4; l++) {
                    const stacks = c.getStackContext(p, ["L" + l]);
                    const st = stacks["L" + l];
                    const items = st ? st.items.map((m) => [c.mergeTree.getPosition(m, 0, c.getClientId()), m.refType]) : [];
                    answers.push([p, l, items]);
                }
            }
            out.push(JSON.stringify({ doc: d, err, len, answers }));
        }
        process.stdout.write(out.join("\n") + "\n");
        return;
    }
    if (mode === "errstate") {
        const out = [];
        for (let d = 0; d < log.nDocs; d++) {
            const msgs = Array.from(messages(log, d));
            let c = newObserver(), err = null, at = -1;
            for (let i = 0; i < msgs.length && err === null; i++) {
                try {
                    c.applyMsg(msgs[i]);
                } catch (e) {
                    err = String(e.message || e);
                    at = i;
                }
            }
            if (err !== null) {
                c = newObserver();
                for (let i = 0; i < at; i++) c.applyMsg(msgs[i]);
            }
            out.push(JSON.stringify({ doc: d, err, err_msg_index: at, err_seq: at >= 0 ? msgs[at].sequenceNumber : null,
                state: canonical(c) }));
        }
        process.stdout.write(out.join("\n") + "\n");
        return;
    }
    if (mode === "snapshot") {
        const d0 = process.argv[4] ? parseInt(process.argv[4], 10) : 0;
        const d1 = Math.min(log.nDocs, process.argv[5] ? parseInt(process.argv[5], 10) : log.nDocs);
        const logger = { send() {}, sendTelemetryEvent() {}, sendErrorEvent() {}, sendPerformanceEvent() {} };
        const out = [];
        for (let d = d0; d < d1; d++) {
            const { c, err } = replayDoc(log, d);
            if (process.argv[6]) {  // mergeTreeSnapshotChunkSize option (snapshotV1.ts:54)
                c.mergeTree.options = Object.assign({}, c.mergeTree.options,
                    { mergeTreeSnapshotChunkSize: parseInt(process.argv[6], 10) });
            }
            const snap = new SnapshotV1(c.mergeTree, logger);
            snap.extractSync();
            const tree = snap.emit();
            const entries = {};
            for (const e of tree.entries) entries[e.path] = JSON.parse(e.value.contents);
            out.push(JSON.stringify({ doc: d, err, snapshot: entries }));
        }
        process.stdout.write(out.join("\n") + "\n");
        return;
    }
    if (mode === "bench") {
        const threads = parseInt(process.argv[4] || "1", 10);
        const file = process.argv[3];
        const t0 = process.hrtime.bigint();
        let done = 0, ops = 0, applyMax = 0;
        for (let t = 0; t < threads; t++) {
            const w = new Worker(__filename, { workerData: { file, t, threads } });
            w.on("message", (m) => {
                ops += m.ops;
                applyMax = Math.max(applyMax, m.apply_ns / 1e9);
                if (++done === threads) {
                    const dt = Number(process.hrtime.bigint() - t0) / 1e9;
                    // apply-only rate: max over workers of the time spent inside applyMsg loops
                    console.log(JSON.stringify({ threads, ops, seconds: dt, ops_per_sec: ops / dt,
                        apply_seconds: applyMax, apply_ops_per_sec: ops / applyMax }));
                }
            });
        }
        return;
    }
    throw new Error("mode: state | errstate | snapshot | load | loadtree | bench");
}

if (isMainThread) {
    main();
} else {
    // worker: docs round-robin (replayMultipleFiles.ts:123-190 pattern); messages pre-built
    // outside the timed loop, as DeltaManager parses JSON upstream (deltaManager.ts:1283-1290)
    const log = loadLog(workerData.file);
    let ops = 0, apply = 0;
    for (let d = workerData.t; d < log.nDocs; d += workerData.threads) {
        const msgs = Array.from(messages(log, d));
        const c = newObserver();
        const t0 = process.hrtime.bigint();
        for (const m of msgs) c.applyMsg(m);
        apply += Number(process.hrtime.bigint() - t0);
        ops += log.rowPtr[d + 1] - log.rowPtr[d];
    }
    parentPort.postMessage({ ops, apply_ns: apply });
}
