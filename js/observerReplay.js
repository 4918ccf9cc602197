"use strict";
// observerReplay.js -- the CPU baseline on the GPU box: a JavaScript restatement of the
// reference's observer apply path (one merge-tree Client per document), run with one
// worker_thread per host core (the pattern of packages/test/snapshots/src/replayMultipleFiles.ts:123-190).
//
// TEST / MEASUREMENT INFRASTRUCTURE ONLY: never on the product path.  The reference itself cannot
// travel to the GPU box, so bench.py times this restatement there and scales it by r, the ratio
// reference / restatement measured in the build container on identical logs
// (oracle/tsref/calibrate.js -> profiles/r02_js_calibration.json).
//
// Restated (same structure as oracle/mtcpu.cpp; the reference functions):
//   Client.applyMsg / updateSeqNumbers         client.ts:797-828
//   insertingWalk / breakTie / split / updateRoot / ensureIntervalBoundary
//                                              mergeTree.ts:2345-2489, 2248-2277, 1876-1887, 2241-2245
//   markRangeRemoved / annotateRange / nodeMap mergeTree.ts:2607-2719, 2565-2605, 2903-2965
//   zamboni: addToLRUSet / zamboniSegments / scourNode / pack   mergeTree.ts:1273-1478
//   Heap                                       collections.ts:213-265
// Block lengths are summed from the leaves (the reference caches them in PartialSequenceLengths).
//
//   node js/observerReplay.js state <log.mtlog>            -> JSON lines {doc, err, state}
//   node js/observerReplay.js bench <log.mtlog> <threads>  -> {ops, threads, apply_seconds, ops_per_sec}
const { Worker, isMainThread, parentPort, workerData } = require("worker_threads");
const { loadLog } = require("./mtlog.js");

const MAX_NODES = 8, TEXT_GRANULARITY = 256, ZAMBONI_MAX = 2;
const INSERT = 0, REMOVE = 1, ANNOTATE = 2, NOOP = 3;
const F_REWRITE = 1, F_PROPS = 2, F_GROUP_MORE = 4, F_MARKER = 128;
const SC_UNDEF = 0, SC_TRUE = 1, SC_FALSE = 2;
const E_SEQ = 1, E_MSN = 2, E_INSERT = 3, E_LIMITS = 6, E_BADOP = 7;

class Seg {
    constructor(text) {
        this.leaf = true; this.parent = undefined; this.text = text;
        this.seq = 0; this.client = 0; this.removed = false; this.rseq = 0; this.rclient = 0;
        this.overlap = 0n; this.props = undefined;  // undefined | array of value ids by key id
        this.marker = false;  // a Marker (mergeTree.ts:630-798): text = its one refType character
    }
}
class Block {
    constructor() { this.leaf = false; this.parent = undefined; this.children = []; this.needsScour = SC_UNDEF; }
}

function segLen(s, R, C) {  // nodeLength leaf branch, mergeTree.ts:1667-1697
    if (s.client === C || s.seq <= R) {
        if (s.removed && (s.rclient === C || ((s.overlap >> BigInt(C)) & 1n) === 1n || s.rseq <= R)) return 0;
        return s.text.length;
    }
    return 0;
}
function nodeLen(n, R, C) {
    if (n.leaf) return segLen(n, R, C);
    let t = 0;
    for (const ch of n.children) t += nodeLen(ch, R, C);
    return t;
}
function breakTie(pos, n, R) {  // mergeTree.ts:2248-2277
    if (!n.leaf) return true;
    if (pos === 0) return !(n.removed && n.rseq <= R);
    return false;
}
function sameProps(a, b) {
    if ((a.props === undefined) !== (b.props === undefined)) return false;
    if (a.props === undefined) return true;
    const n = Math.max(a.props.length, b.props.length);
    for (let k = 0; k < n; k++) if ((a.props[k] || 0) !== (b.props[k] || 0)) return false;
    return true;
}

class Doc {
    constructor() {
        this.root = new Block(); this.currentSeq = 0; this.minSeq = 0;
        this.heap = [{ seg: undefined, maxSeq: -2 }]; this.err = 0; this.errSeq = 0;
    }
    fail(code, seq) { if (!this.err) { this.err = code; this.errSeq = seq; } }

    split(node) {  // mergeTree.ts:2476-2489
        const nb = new Block();
        nb.children = node.children.splice(MAX_NODES / 2);
        for (const ch of nb.children) ch.parent = nb;
        return nb;
    }
    updateRoot(sp) {  // mergeTree.ts:1876-1887
        if (!sp) return;
        const nr = new Block();
        nr.children = [this.root, sp];
        this.root.parent = nr; sp.parent = nr;
        this.root = nr;
    }
    splitAt(s, pos) {  // BaseSegment.splitAt + TextSegment.createSplitSegmentAt
        const r = new Seg(s.text.substring(pos));
        s.text = s.text.substring(0, pos);
        r.props = s.props === undefined ? undefined : s.props.slice();
        r.removed = s.removed; r.rseq = s.rseq; r.rclient = s.rclient; r.seq = s.seq; r.client = s.client;
        r.overlap = s.overlap; r.marker = s.marker;
        return r;
    }
    insertingWalk(b, pos, R, C, cand) {  // mergeTree.ts:2345-2474
        let ci = 0, newNode;
        for (; ci < b.children.length; ci++) {
            const child = b.children[ci];
            const len = nodeLen(child, R, C);
            if (pos < len || (pos === len && breakTie(pos, child, R))) {
                if (!child.leaf) {
                    const sp = this.insertingWalk(child, pos, R, C, cand);
                    if (!sp) return undefined;
                    newNode = sp; ci++;
                } else if (cand) {
                    b.children[ci] = cand; cand.parent = b;
                    newNode = child; ci++;
                } else {
                    if (!(pos > 0)) return undefined;
                    newNode = this.splitAt(child, pos); ci++;
                }
                break;
            } else {
                pos -= len;
            }
        }
        if (!newNode && pos === 0 && cand) newNode = cand;
        if (!newNode) return undefined;
        b.children.splice(ci, 0, newNode);
        newNode.parent = b;
        if (b.children.length < MAX_NODES) return undefined;
        return this.split(b);
    }
    ensureIntervalBoundary(pos, R, C) { this.updateRoot(this.insertingWalk(this.root, pos, R, C, undefined)); }

    heapAdd(x) {
        const h = this.heap;
        h.push(x);
        let k = h.length - 1;
        while (k > 1 && h[k >> 1].maxSeq - h[k].maxSeq > 0) {
            const t = h[k >> 1]; h[k >> 1] = h[k]; h[k] = t; k >>= 1;
        }
    }
    heapGet() {
        const h = this.heap, x = h[1];
        h[1] = h[h.length - 1];
        h.pop();
        const count = h.length - 1;
        let k = 1;
        while ((k << 1) <= count) {
            let j = k << 1;
            if (j < count && h[j].maxSeq - h[j + 1].maxSeq > 0) j++;
            if (h[k].maxSeq - h[j].maxSeq <= 0) break;
            const t = h[k]; h[k] = h[j]; h[j] = t; k = j;
        }
        return x;
    }
    addToLRUSet(s, seq) {  // mergeTree.ts:1273-1283
        if (s.parent.needsScour !== SC_TRUE && seq > this.currentSeq) {
            s.parent.needsScour = SC_TRUE;
            this.heapAdd({ seg: s, maxSeq: seq });
        }
    }
    scourNode(node, hold) {  // mergeTree.ts:1289-1365
        let prev;
        for (const child of node.children) {
            if (!child.leaf) { hold.push(child); prev = undefined; continue; }
            const s = child;
            if (s.removed) {
                if (s.rseq > this.minSeq) hold.push(s); else s.parent = undefined;
                prev = undefined;
            } else if (s.seq <= this.minSeq) {
                const app = prev && !prev.marker && !s.marker && !prev.text.endsWith("\n") &&
                    (prev.text.length <= TEXT_GRANULARITY || s.text.length <= TEXT_GRANULARITY) &&
                    sameProps(prev, s) && s.text.length > 0;
                if (app) {
                    prev.text += s.text;
                    s.parent = undefined;
                } else {
                    hold.push(s);
                    prev = s.text.length > 0 ? s : undefined;
                }
            } else {
                hold.push(s); prev = undefined;
            }
        }
    }
    pack(block) {  // mergeTree.ts:1368-1420
        const parent = block.parent, hold = [];
        for (const cb of parent.children) { this.scourNode(cb, hold); cb.parent = undefined; }
        const total = hold.length;
        let cc = Math.min(MAX_NODES - 1, Math.floor(total / (MAX_NODES / 2)));
        if (cc < 1) cc = 1;
        const base = Math.floor(total / cc);
        let extra = total % cc, rd = 0;
        const packed = [];
        for (let ni = 0; ni < cc; ni++) {
            let nc = base;
            if (extra > 0) { nc++; extra--; }
            const pb = new Block();
            pb.children = hold.slice(rd, rd + nc);
            rd += nc;
            for (const ch of pb.children) ch.parent = pb;
            pb.parent = parent;
            packed.push(pb);
        }
        parent.children = packed;
        if (parent.children.length < MAX_NODES / 2 && parent.parent) this.pack(parent);
    }
    zamboni() {  // mergeTree.ts:1422-1478
        for (let i = 0; i < ZAMBONI_MAX; i++) {
            if (this.heap.length <= 1 || this.heap[1].maxSeq > this.minSeq) break;
            const s = this.heapGet().seg;
            if (s.parent && s.parent.needsScour !== SC_FALSE) {
                const b = s.parent, hold = [];
                this.scourNode(b, hold);
                b.needsScour = SC_FALSE;
                if (hold.length < b.children.length) {
                    b.children = hold;
                    for (const ch of hold) ch.parent = b;
                    if (b.children.length < MAX_NODES / 2 && b.parent) this.pack(b);
                }
            }
        }
    }
    nodeMap(node, R, C, start, end, leaf) {  // mergeTree.ts:2903-2965
        for (const child of node.children.slice()) {
            const len = nodeLen(child, R, C);
            if (end > 0 && len > 0 && start < len) {
                if (!child.leaf) this.nodeMap(child, R, C, start, end, leaf); else leaf(child);
            }
            start -= len;
            end -= len;
        }
    }
    apply(r, text, pairs, last) {  // Client.applyMsg for one record (client.ts:797-828)
        if (this.err) return;
        const S = r.seq, R = r.ref, C = r.client;
        if (r.type > NOOP) return this.fail(E_BADOP, S);
        if (r.type !== NOOP) {
            if (C >= 64 || C === 0) return this.fail(E_LIMITS, S);
            let wc = 0;
            if (!(this.currentSeq < S)) wc = E_SEQ;
            else if (!(this.minSeq <= r.msn) || !(r.msn <= S)) wc = E_MSN;
            if (wc) {
                if (r.type === INSERT && text.length > 0 && r.pos1 > nodeLen(this.root, R, C)) wc = E_INSERT;
                return this.fail(wc, S);
            }
        } else {
            if (!(this.currentSeq <= S)) return this.fail(E_SEQ, S);
            if (!(r.msn <= S) || !(this.minSeq <= r.msn)) return this.fail(E_MSN, S);
        }
        if (r.type === INSERT) {
            if (r.pos1 < 0) return this.fail(E_BADOP, S);
            this.ensureIntervalBoundary(r.pos1, R, C);
            if (text.length > 0) {
                const s = new Seg(text);
                if (r.flags & F_PROPS) {
                    s.props = [];
                    for (let q = 0; q < pairs.length; q += 2) s.props[pairs[q]] = pairs[q + 1];
                }
                s.seq = S; s.client = C; s.marker = (r.flags & F_MARKER) !== 0;
                const sp = this.insertingWalk(this.root, r.pos1, R, C, s);
                if (!s.parent) return this.fail(E_INSERT, S);
                this.updateRoot(sp);
                if (S > this.minSeq) this.addToLRUSet(s, S);
            }
            this.zamboni();
        } else if (r.type === REMOVE || r.type === ANNOTATE) {
            if (r.pos1 < 0 || r.pos2 < 0) return this.fail(E_BADOP, S);
            this.ensureIntervalBoundary(r.pos1, R, C);
            this.ensureIntervalBoundary(r.pos2, R, C);
            if (r.type === REMOVE) {
                const cbit = 1n << BigInt(C);
                this.nodeMap(this.root, R, C, r.pos1, r.pos2, (s) => {
                    if (s.removed) s.overlap |= cbit;
                    else { s.removed = true; s.rseq = S; s.rclient = C; }
                    this.addToLRUSet(s, S);
                });
            } else {
                const rewrite = (r.flags & F_REWRITE) !== 0;
                this.nodeMap(this.root, R, C, r.pos1, r.pos2, (s) => {
                    if (s.props === undefined || rewrite) s.props = [];
                    for (let q = 0; q < pairs.length; q += 2) s.props[pairs[q]] = pairs[q + 1];
                    this.addToLRUSet(s, S);
                });
            }
            this.zamboni();
        }
        if (last) {  // updateSeqNumbers (client.ts:821-828), setMinSeq (mergeTree.ts:1718-1736)
            this.currentSeq = S;
            if (r.msn > this.minSeq) { this.minSeq = r.msn; this.zamboni(); }
        }
    }
    canonical() {  // DESIGN.md "Canonical state"
        const segs = [];
        const walk = (n) => {
            if (n.leaf) {
                const ov = [];
                for (let c = 0; c < 64; c++) if ((n.overlap >> BigInt(c)) & 1n) ov.push(c);
                let props = null;
                if (n.props !== undefined) {
                    props = {};
                    n.props.forEach((v, k) => { if (v) props["k" + k] = v; });
                }
                segs.push([n.marker ? { marker: n.text.charCodeAt(0) } : n.text, n.seq, n.client,
                    n.removed ? n.rseq : -1, n.removed ? n.rclient : -1, ov, props]);
                return;
            }
            for (const ch of n.children) walk(ch);
        };
        walk(this.root);
        const tree = [];
        let lvl = [this.root];
        while (lvl.length) {
            tree.push(lvl.map((b) => b.children.length));
            const nxt = [];
            for (const b of lvl) for (const ch of b.children) if (!ch.leaf) nxt.push(ch);
            lvl = nxt;
        }
        return { seq: this.currentSeq, msn: this.minSeq, segs, tree };
    }
}

// the records of document d, decoded once (outside any timed loop, as DeltaManager parses upstream)
function records(log, d) {
    const b = log.buf, out = [];
    for (let i = log.rowPtr[d]; i < log.rowPtr[d + 1]; i++) {
        const o = log.opsOff + 32 * i;
        const r = { seq: b.readInt32LE(o), ref: b.readInt32LE(o + 4), msn: b.readInt32LE(o + 8),
            client: b.readUInt16LE(o + 12), type: b.readUInt8(o + 14), flags: b.readUInt8(o + 15),
            pos1: b.readInt32LE(o + 16), pos2: b.readInt32LE(o + 20) };
        const poff = log.payOff + b.readUInt32LE(o + 24), plen = b.readUInt32LE(o + 28);
        const np = (r.flags >> 3) & 15;
        const text = b.toString("latin1", poff, poff + plen - 2 * np);
        const pairs = [];
        for (let q = 0; q < 2 * np; q++) pairs.push(b.readUInt8(poff + plen - 2 * np + q));
        out.push([r, text, pairs, !(r.flags & F_GROUP_MORE)]);
    }
    return out;
}

function replay(recs) {
    const doc = new Doc();
    for (const [r, text, pairs, last] of recs) doc.apply(r, text, pairs, last);
    return doc;
}

function main() {
    const mode = process.argv[2], file = process.argv[3];
    if (mode === "state") {
        const log = loadLog(file), out = [];
        for (let d = 0; d < log.nDocs; d++) {
            const doc = replay(records(log, d));
            out.push(JSON.stringify({ doc: d, err: doc.err ? [doc.err, doc.errSeq] : null, state: doc.canonical() }));
        }
        process.stdout.write(out.join("\n") + "\n");
        return;
    }
    if (mode === "bench") {
        const threads = parseInt(process.argv[4] || "1", 10);
        let done = 0, ops = 0, applyMax = 0;
        for (let t = 0; t < threads; t++) {
            const w = new Worker(__filename, { workerData: { file, t, threads } });
            w.on("message", (m) => {
                ops += m.ops;
                applyMax = Math.max(applyMax, m.apply_ns / 1e9);
                if (++done === threads) {
                    console.log(JSON.stringify({ ops, threads, apply_seconds: applyMax, ops_per_sec: ops / applyMax }));
                }
            });
        }
        return;
    }
    throw new Error("mode: state | bench");
}

if (isMainThread) {
    main();
} else {
    // documents round-robin over the workers; each times only its applies
    const log = loadLog(workerData.file);
    let ops = 0, apply = 0;
    for (let d = workerData.t; d < log.nDocs; d += workerData.threads) {
        const recs = records(log, d);
        const t0 = process.hrtime.bigint();
        replay(recs);
        apply += Number(process.hrtime.bigint() - t0);
        ops += recs.length;
    }
    parentPort.postMessage({ ops, apply_ns: apply });
}

module.exports = { Doc, records, replay };
