"use strict";
// A multi-client farm over the REFERENCE merge-tree Clients (type-stripped into oracle/_tsref) that
// writes op logs seen from one editing client: the client under test ("c1") makes local edits
// (insertSegmentLocal / removeRangeLocal / annotateRangeLocal, client.ts:163-214) while the other
// clients edit concurrently; a toy sequencer orders every client's messages (msn = the least
// seq any client may still reference: its currentSeq or an in-flight op's refSeq) and each client receives the sequenced stream at its own pace, so
// c1's own messages come back as acks (client.ts:588-625, 804-806) interleaved with remote ops.
// The pattern of client.conflictFarm.spec.ts / mergeTreeOperationRunner.ts; with `partial` c1 also
// lags behind the stream.  A run whose clients end with different text is dropped (the reference
// itself diverges on some lagging-client runs; such logs are not used as fixtures).
// TEST INFRASTRUCTURE ONLY (this container).
//   node local_farm.js <nDocs> <seed> <opsPerDoc> [nClients [partial [markers [reconnect [offline]]]]] -> JSON {docs: [[record, ...], ...]}
//   record = [seq, ref, msn, client, type, pos1, pos2, text, props {key id: value id | null} | null,
//             flags]; c1's local edits have seq = -1 (UnassignedSequenceNumber), ref = msn = 0
const path = require("path");
const ROOT = path.join(__dirname, "..", "_tsref", "merge-tree", "src");
const { Client } = require(path.join(ROOT, "client.js"));
const { TextSegment } = require(path.join(ROOT, "textSegment.js"));
const { Marker } = require(path.join(ROOT, "mergeTree.js"));

function specToSegment(spec) { return TextSegment.fromJSONObject(spec) || Marker.fromJSONObject(spec); }
const logger = { send() {}, sendTelemetryEvent() {}, sendErrorEvent() {}, sendPerformanceEvent() {} };

function rng(seed) {  // xorshift32
    let s = seed >>> 0 || 1;
    return () => {
        s ^= s << 13; s >>>= 0; s ^= s >>> 17; s ^= s << 5; s >>>= 0;
        return s / 4294967296;
    };
}

const F_REWRITE = 1, F_MARKER = 128;
// one record per op; a GROUP op as its members (all but the last flagged "more"), an empty GROUP
// as a no-op record
const F_GROUP_MORE = 4;
function records(seq, ref, msn, client, op) {
    if (op.type !== 3) return [record(seq, ref, msn, client, op)];
    if (!op.ops.length) return [[seq, ref, msn, client, 3, 0, 0, null, null, 0]];
    return op.ops.map((m, i) => {
        const r = record(seq, ref, msn, client, m);
        if (i + 1 < op.ops.length) r[9] |= F_GROUP_MORE;
        return r;
    });
}
function record(seq, ref, msn, client, op) {
    const props = (p) => {
        if (!p) return null;
        const o = {};
        for (const k of Object.keys(p)) o[parseInt(k.slice(1), 10)] = p[k] === null || p[k] === undefined ? null : p[k];
        return o;
    };
    if (op.type === 0) {
        const seg = op.seg;
        if (seg.marker) {  // IJSONMarkerSegment: the record's one text byte is its refType
            return [seq, ref, msn, client, 0, op.pos1, 0, String.fromCharCode(seg.marker.refType), props(seg.props),
                F_MARKER];
        }
        const text = typeof seg === "string" ? seg : seg.text;
        return [seq, ref, msn, client, 0, op.pos1, 0, text, typeof seg === "string" ? null : props(seg.props), 0];
    }
    if (op.type === 1) return [seq, ref, msn, client, 1, op.pos1, op.pos2, null, null, 0];
    return [seq, ref, msn, client, 2, op.pos1, op.pos2, null, props(op.props),
        op.combiningOp && op.combiningOp.name === "rewrite" ? F_REWRITE : 0];
}

function farm(seed, nOps, nClients, partial, markers, reconnect, offline) {
    const r = rng(seed);
    const ri = (n) => Math.floor(r() * n);
    const clients = [];
    for (let i = 1; i <= nClients; i++) {
        const c = new Client(specToSegment, logger);
        c.startOrUpdateCollaboration("c" + i);
        clients.push(c);
    }
    const queue = [];      // submitted, not yet sequenced: {client, ref, op}
    const seqd = [];       // sequenced messages
    const cursor = clients.map(() => 0);
    const log = [];        // c1's view
    const regen = [];      // [index of the seq -2 record, regenerated ops]
    let seq = 0, made = 0;
    let away = 0;          // offline: rounds c1 still stays offline (its messages held, nothing delivered)
    const deliver = (i) => {
        const m = seqd[cursor[i]++];
        clients[i].applyMsg(m);
        if (i === 0) log.push(...records(m.sequenceNumber, m.referenceSequenceNumber, m.minimumSequenceNumber,
            parseInt(m.clientId.slice(1), 10), m.contents));
    };
    const localOp = (i) => {
        const c = clients[i];
        const len = c.getLength();
        const pick = r();
        let op;
        if (len === 0 || pick < 0.45) {
            const n = 1 + ri(4);
            let text = "";
            for (let q = 0; q < n; q++) text += String.fromCharCode(97 + ri(26));
            let props;
            if (r() < 0.25) { props = {}; props["k" + ri(3)] = 1 + ri(4); }
            const seg = markers && r() < 0.15 ? new Marker([1, 2, 4][ri(3)]) : new TextSegment(text);
            if (props) seg.addProperties(props);
            op = c.insertSegmentLocal(ri(len + 1), seg);
        } else {
            const a = ri(len), b = a + 1 + ri(Math.min(6, len - a));
            if (pick < 0.75) {
                op = c.removeRangeLocal(a, b);
            } else {
                const props = {};
                const nk = 1 + ri(2);
                for (let q = 0; q < nk; q++) props["k" + ri(3)] = r() < 0.15 ? null : 1 + ri(4);
                op = c.annotateRangeLocal(a, b, props, r() < 0.1 ? { name: "rewrite" } : undefined);
            }
        }
        if (!op) throw new Error("local op rejected");
        // (the pending group of the edit: what regeneratePendingOp is handed on reconnect)
        queue.push({ client: i + 1, ref: c.getCurrentSeq(), op, sg: c.peekPendingSegmentGroups() });
        if (i === 0) log.push(record(-1, 0, 0, 1, op));
        made++;
    };
    const sequenceAll = (hold) => {
        const held = [];   // (hold: c1 is offline, its messages wait in order)
        while (queue.length) {
            const q = queue.shift();
            if (hold && q.client === 1) {
                held.push(q);
                continue;
            }
            seq++;
            // no client may still reference a seq below the msn: its in-flight ops included
            const msn = Math.min(q.ref, ...clients.map((c) => c.getCurrentSeq()), ...queue.map((o) => o.ref),
                                 ...held.map((o) => o.ref));
            seqd.push({ clientId: "c" + q.client, clientSequenceNumber: 1, contents: q.op, metadata: undefined,
                minimumSequenceNumber: msn, origin: undefined, referenceSequenceNumber: q.ref, sequenceNumber: seq,
                timestamp: 0, term: 1, traces: [], type: "op" });
        }
        queue.push(...held);
    };
    // rounds (mergeTreeOperationRunner.ts): clients edit, the round's ops are sequenced, and every
    // client catches up -- c1 only to a random point when `partial`, so its next edits interleave
    // with the rest of the stream
    while (made < nOps) {
        // offline: now and then c1 goes offline for 12-24 rounds, editing more per round; its
        // messages are held (so its pending edits pile up past 64) and it receives nothing
        // (offline 2: long sessions, 90-120 rounds at 3-7 edits each, so 400+ of c1's edits are
        // pending at once -- capped at 480)
        if (offline && !away && r() < (offline === 2 ? 0.05 : 0.08)) away = offline === 2 ? 90 + ri(31) : 12 + ri(13);
        for (let i = 0; i < nClients; i++) {
            let k = away && i === 0 ? (offline === 2 ? 3 + ri(5) : 1 + ri(5)) : r() < 0.6 ? 1 + ri(3) : 0;
            if (away && i === 0 && offline === 2) k = Math.min(k, 480 - queue.filter((q) => q.client === 1).length);
            for (let q = 0; q < k; q++) localOp(i);
        }
        // reconnect (client.reconnectFarm.spec.ts): c1's messages of this round are never sequenced;
        // c1 catches up with everything else, then regenerates each lost op (regeneratePendingOp,
        // client.ts:855-893) and submits the new one.  In c1's log: one record with seq -2 per lost
        // op (the op being reset), and the regenerated ops in `regen`
        let lost = [];
        if (reconnect && r() < 0.5) {
            lost = queue.filter((q) => q.client === 1);
            for (let q = queue.length - 1; q >= 0; q--) if (queue[q].client === 1) queue.splice(q, 1);
        }
        sequenceAll(away > 0);
        for (let i = 1; i < nClients; i++) while (cursor[i] < seqd.length) deliver(i);
        if (away) {
            away--;
            continue;
        }
        const upto = partial ? cursor[0] + ri(seqd.length - cursor[0] + 1) : seqd.length;
        while (cursor[0] < upto) deliver(0);
        for (const q of lost) {
            const c = clients[0];
            log.push(...records(-2, 0, 0, 1, q.op));
            const op = c.regeneratePendingOp(q.op, q.sg);
            regen.push([log.length - 1, (op.type === 3 ? op.ops : [op]).map((m) => record(0, 0, 0, 1, m).slice(4))]);
            queue.push({ client: 1, ref: c.getCurrentSeq(), op, sg: undefined });
        }
        if (lost.length) {  // the regenerated ops are sequenced and reach everyone in the same round
            sequenceAll();
            for (let i = 0; i < nClients; i++) while (cursor[i] < seqd.length) deliver(i);
        }
    }
    if (offline === 2 && queue.length) {  // (a long session may outlast the edits: c1 comes back at the end)
        sequenceAll(false);
        for (let i = 1; i < nClients; i++) while (cursor[i] < seqd.length) deliver(i);
    }
    while (cursor[0] < seqd.length) deliver(0);
    const txt = (c) => c.createTextHelper().getText(c.getCurrentSeq(), c.getClientId());
    const t0 = txt(clients[0]);
    for (const c of clients) if (txt(c) !== t0) {  // the clients diverged: drop the run
        if (process.env.FARM_DEBUG) process.stderr.write(`local_farm: diverged (${clients.map((x) => txt(x).length)})\n`);
        return null;
    }
    return reconnect ? { log, regen } : log;
}

const [nDocs, seed, nOps, nClients, partial, markers, reconnect, offline] =
    process.argv.slice(2).map((x) => parseInt(x, 10));
const docs = [];
let dropped = 0;
for (let d = 0, k = 0; d < nDocs; k++) {
    let log = null;
    try {  // (offline runs: a reference client may throw "MergeTree insert failed" -- dropped like a divergence)
        log = farm(seed * 7919 + k, nOps, nClients || 4, partial === 1, markers === 1, reconnect === 1,
                   offline || 0);
    } catch (err) {
        if (!offline) throw err;
        if (process.env.FARM_DEBUG && dropped < 5) process.stderr.write(`local_farm: run ${k}: ${err.message}\n`);
    }
    if (log) { docs.push(log); d++; } else dropped++;
    if (offline === 2 && k % 10 === 9) process.stderr.write(`local_farm: ${k + 1} runs, ${dropped} dropped\n`);
}
process.stderr.write(`local_farm: ${nDocs} documents, ${dropped} runs dropped (clients diverged)\n`);
process.stdout.write(JSON.stringify({ docs }) + "\n");
