"use strict";
// Observer-driven op logs beyond the narrow device limits (include/mtgpu.h "limits"), generated over
// the REFERENCE merge-tree (type-stripped into oracle/_tsref): many client ids (> 100 per document),
// UTF-16 text (CJK, surrogate pairs -- inserts and removes that split them), property value ids past
// 255 and keys past 7.  As in the synthetic model (DESIGN.md "Synthetic workloads"): op i picks a
// client C and a refSeq R (lag <= maxLag behind the last seq, never below C's last R), and its
// positions inside getLength(R, C) of the reference observer (mergeTree.ts:1577), so every op is
// valid for what C had seen; the observer then applies it (Client.applyMsg).
// TEST INFRASTRUCTURE ONLY (this container).
//   node wide_log.js <nDocs> <seed> <opsPerDoc> <nClients> [maxLag] -> JSON {docs: [[record, ...], ...]}
//   record = [seq, ref, msn, client, type, pos1, pos2, text, props {key id: value id | null} | null, flags]
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

// text pieces: ASCII, Latin-1, CJK, emoji (surrogate pairs), newlines
const PIECES = ["a", "b", "z", "0", "7", " ", "é", "ü", "中", "文", "字", "Ж",
    "😀", "🎉", "𝄞", "\n"];

function main() {
    const [nDocs, seed, opsPerDoc, nClients] = process.argv.slice(2, 6).map((x) => parseInt(x, 10));
    const maxLag = parseInt(process.argv[6] || "8", 10);
    // property keys: annotates draw keys 0..nKeys-5 (0..11 at the default 16) and a second key from
    // all nKeys; inserts the first range
    const nKeys = parseInt(process.argv[7] || "16", 10), k1 = nKeys === 16 ? 11 : nKeys - 5;
    const docs = [];
    for (let d = 0; d < nDocs; d++) {
        const r = rng(seed * 7919 + d * 104729 + 1);
        const u = (lo, hi) => lo + Math.floor(r() * (hi - lo + 1));
        const obs = new Client(specToSegment, logger);
        obs.startOrUpdateCollaboration("observer");
        const lastRef = new Array(nClients + 1).fill(0);
        const recs = [];
        let seq = 0;
        for (let i = 0; i < opsPerDoc; i++) {
            // clients join over time: the first ops use few ids, later ones all of them
            const C = u(1, Math.max(2, Math.min(nClients, 4 + Math.floor((i * nClients) / (opsPerDoc / 2)))));
            const R = Math.max(lastRef[C], seq - u(0, maxLag));
            lastRef[C] = R;
            let msn = seq;  // the least refSeq any active client may still send: here the window's lower end
            for (let c = 1; c <= nClients; c++) msn = Math.min(msn, Math.max(lastRef[c], seq - maxLag));
            msn = Math.max(0, Math.min(msn, R));
            // the log's short id: client C, past 253 one up (254 is NonCollabClient's in the engine's
            // log form, include/mtgpu.h)
            const id = C < 254 ? C : C + 1;
            const shortId = obs.getOrAddShortClientId("c" + id);
            const L = obs.mergeTree.getLength(R, shortId);
            const t = r();
            let rec;
            const S = seq + 1;
            if (t < 0.5 || L === 0) {
                let text = "";
                for (let n = u(1, 6); n > 0; n--) text += PIECES[u(0, PIECES.length - 1)];
                let props = null;
                if (r() < 0.25) {
                    props = {};
                    props[u(0, k1)] = u(1, 1200);
                }
                rec = [S, R, msn, id, 0, u(0, L), 0, text, props, 0];
            } else {
                const a = u(0, L - 1), b = Math.min(L, a + u(1, 8));
                if (t < 0.78) {
                    rec = [S, R, msn, id, 1, a, b, null, null, 0];
                } else {
                    const props = {};
                    props[u(0, k1)] = r() < 0.1 ? null : u(1, 1500);
                    if (r() < 0.4) props[u(0, nKeys - 1)] = u(1, 400);
                    rec = [S, R, msn, id, 2, a, b, null, props, r() < 0.05 ? 1 : 0];
                }
            }
            const op = toOp(rec);
            obs.applyMsg({ clientId: "c" + id, clientSequenceNumber: 1, contents: op, metadata: undefined,
                minimumSequenceNumber: msn, origin: undefined, referenceSequenceNumber: R, sequenceNumber: S,
                timestamp: 0, term: 1, traces: [], type: "op" });
            seq = S;
            recs.push(rec);
        }
        docs.push(recs);
    }
    process.stdout.write(JSON.stringify({ docs }) + "\n");
}

function toOp(rec) {
    const [, , , , type, p1, p2, text, props, flags] = rec;
    const kp = (p) => {
        if (!p) return undefined;
        const o = {};
        for (const k of Object.keys(p)) o["k" + k] = p[k];
        return o;
    };
    if (type === 0) return { type: 0, pos1: p1, seg: props ? { text, props: kp(props) } : text };
    if (type === 1) return { type: 1, pos1: p1, pos2: p2 };
    const op = { type: 2, pos1: p1, pos2: p2, props: kp(props) };
    if (flags & 1) op.combiningOp = { name: "rewrite" };
    return op;
}

main();
