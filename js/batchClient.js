"use strict";
// batchClient.js -- the reference's op-apply surface over the MI355X engine (CommonJS, node 12).
//
// BatchClient mirrors the observer `Client` of packages/dds/merge-tree/src/client.ts:
//   applyMsg(msg)                       client.ts:797-819   (queued; applied in device batches)
//   startOrUpdateCollaboration(longId)  client.ts:1051-1071
//   getLength() / getCurrentSeq()       client.ts:1042-1049
// plus the TestClient helpers of src/test/testClient.ts:102-234 (getText, makeOpMessage,
// insertTextRemote, removeRangeRemote, enqueueMsg, applyMessages).  Many BatchClients share one
// BatchEngine (one MI355X); any read flushes every client's queued ops as ONE batched submit.
// An editing client's local edits (insertTextLocal / insertMarkerLocal / removeRangeLocal /
// annotateRangeLocal) apply on the device in its local view, its own sequenced messages ack them,
// and regeneratePendingOp serves a reconnect; register ops and combining ops other than "rewrite"
// throw.
// Delta / maintenance callbacks (mergeTreeDeltaCallback.ts:15-73): setting a client's
// mergeTreeDeltaCallback or mergeTreeMaintenanceCallback makes the engine record them
// (mt_events_enable); they are delivered, in firing order, after the batch that fired them --
// or, with `new BatchEngine({ syncCallbacks: true })`, before applyMsg / the local edit that fired them
// returns: a client with callbacks then flushes per message (per member of a GROUP op, b = 1 for its
// document), so a listener reading getText() / getLength() / getPosition(deltaSegment.segment) inside
// its callback sees what the reference's listener sees (mergeTree.ts:1981-1988: the op applied; the
// text and lengths are those zamboni leaves unchanged; a delta segment's position is the one at
// callback time).  Maintenance callbacks (SPLIT / APPEND / UNLINK) are delivered the same way, after
// the message (a SPLIT's listener reads the text with the op applied).
// Segments are identified by position: deltaSegments[i].segment = {ordinal, position,
// cachedLength} (ordinal among the linked leaves at callback time; position in the local view,
// op callbacks only) -- include/mtgpu.h "delta / maintenance events".
const path = require("path");

const native = require(path.join(__dirname, "mtgpu.node"));

const INSERT = 0, REMOVE = 1, ANNOTATE = 2, GROUP = 3, NOOP = 3;
const F_REWRITE = 1, F_PROPS = 2, F_GROUP_MORE = 4, F_MARKER = 128;
const OP_WIDE = 0x80;  // MT_OP_WIDE: UTF-16 text, (key u8, value u16) pairs
const OP_NP16 = 0x40;  // MT_OP_NP16: property pair count bit 4 (wide records)
const OP_NP32 = 0x20;  // MT_OP_NP32: property pair count bit 5 (wide records)
// mt_pos_query (include/mtgpu.h): kinds, and the local view's refSeq
const POS_CONTAINING = 0, POS_OF_ORDINAL = 1, POS_LOCAL = -2147483648;
// include/mtgpu.h "limits": the wide form's (a document goes wide with its first op beyond the narrow
// ones: client id >= 64, key >= 8, value id >= 256 or a code unit above U+00FF)
const MAX_CLIENTS = 65535, NONCOLLAB_ID = 0xfe, MAX_KEYS = 32, MAX_VALUES = 65535, NARROW_CLIENTS = 64, NARROW_KEYS = 8;
const REC = 32, EVREC = 96, OVX_IDS = 32;  // (MT_OVX_IDS)

function canonicalJson(v) {
    if (Array.isArray(v)) return "[" + v.map(canonicalJson).join(",") + "]";
    if (v !== null && typeof v === "object") {
        return "{" + Object.keys(v).sort().map((k) => JSON.stringify(k) + ":" + canonicalJson(v[k])).join(",") + "}";
    }
    return JSON.stringify(v);
}

class BatchEngine {
    constructor(opts = {}) {
        this.maxDocs = opts.maxDocs || 1;
        this.handle = native.createEngine({
            device: opts.device || 0, maxDocs: this.maxDocs, opsPerLaunch: opts.opsPerLaunch || 0,
            segCapacity: opts.segCapacity || 0, textCapacity: opts.textCapacity || 0,
        });
        this.clients = [];
        this.pending = 0;
        this.recording = false;
        this.eventsPerDoc = opts.eventsPerDoc || (1 << 16);
        this.labelDecl = [];  // [doc, tile key, range key] to declare before the next submit
        this.gen = 0;         // bumped by every submit: segment descriptors are valid within one generation
        this.syncCallbacks = !!opts.syncCallbacks;  // deliver callbacks before the firing call returns
        this.delivering = false;
    }

    _enableEvents() {
        if (this.recording) return;
        this.flush();  // ops queued before the callback was set were "applied" before it
        native.eventsEnable(this.handle, this.eventsPerDoc);
        this.recording = true;
    }

    /** Deliver the callbacks recorded so far to each client (mt_events_drain). */
    _dispatch() {
        if (!this.recording) return;
        const [rows, rpBuf] = native.eventsDrain(this.handle, this.maxDocs);
        const rp = new Uint32Array(rpBuf.buffer, rpBuf.byteOffset, this.maxDocs + 1);
        this.delivering = true;
        try {
            for (let d = 0; d < this.clients.length; d++) {
                if (rp[d + 1] > rp[d]) this.clients[d]._deliver(rows, rp[d], rp[d + 1]);
            }
        } finally {
            this.delivering = false;
        }
        // (ops a listener queued while the callbacks ran: applied now, their callbacks delivered in turn)
        if (this.syncCallbacks && this.pending) this.flush();
    }
    /** syncCallbacks: a client with callbacks applies what it queued before the firing call returns. */
    _syncPoint(client) {
        if (this.syncCallbacks && this.recording && !this.delivering && (client._delta || client._maintenance)) this.flush();
    }

    createClient() {
        if (this.clients.length >= this.maxDocs) throw new Error("BatchEngine: maxDocs reached");
        const c = new BatchClient(this, this.clients.length);
        this.clients.push(c);
        return c;
    }

    _encode() {
        for (const [doc, tk, rk] of this.labelDecl) native.setLabelKeys(this.handle, doc, tk, rk);
        this.labelDecl = [];
        this.gen++;
        const n = this.maxDocs;
        const rowPtr = new Uint32Array(n + 1);
        let nops = 0, nbytes = 0;
        for (let d = 0; d < n; d++) {
            const c = this.clients[d];
            if (c) for (const r of c.queue) { nops++; nbytes += r.payload.length; }
            rowPtr[d + 1] = nops;
        }
        const ops = Buffer.alloc(nops * REC);
        const payload = Buffer.alloc(Math.max(1, nbytes));
        let i = 0, off = 0;
        for (let d = 0; d < n; d++) {
            const c = this.clients[d];
            if (!c) continue;
            for (const r of c.queue) {
                const o = i * REC;
                ops.writeInt32LE(r.seq, o); ops.writeInt32LE(r.ref, o + 4); ops.writeInt32LE(r.msn, o + 8);
                ops.writeUInt16LE(r.client, o + 12);
                // 16..32 pairs (wide only): the count's bits 4 / 5 are type bits 6 / 5 (include/mtgpu.h
                // MT_OP_NP16 / MT_OP_NP32)
                if (r.npairs > MAX_KEYS) throw new Error(`BatchClient: more than ${MAX_KEYS} property pairs in one op`);
                ops.writeUInt8(r.type | ((r.npairs & 16) ? OP_NP16 : 0) | ((r.npairs & 32) ? OP_NP32 : 0), o + 14);
                ops.writeUInt8(r.flags | ((r.npairs & 15) << 3), o + 15);
                ops.writeInt32LE(r.pos1, o + 16); ops.writeInt32LE(r.pos2, o + 20);
                ops.writeUInt32LE(off, o + 24); ops.writeUInt32LE(r.payload.length, o + 28);
                r.payload.copy(payload, off);
                off += r.payload.length;
                i++;
            }
            c.queue = [];
        }
        this.pending = 0;
        return { ops, payload, rowPtr };
    }

    /** Apply every queued op of every client (one device batch). */
    flush() {
        if (!this.pending) return;
        const { ops, payload, rowPtr } = this._encode();
        native.submit(this.handle, ops, payload, rowPtr);
        this._dispatch();
    }

    /** The same as a Promise (napi_async_work): the JS thread stays free while the GPU applies. */
    flushAsync() {
        if (!this.pending) return Promise.resolve();
        const b = this._encode();
        return native.submitAsync(this.handle, b.ops, b.payload, b.rowPtr).then(() => this._dispatch());
    }
}

class BatchClient {
    constructor(engine, doc) {
        this.engine = engine;
        this.doc = doc;
        this.queue = [];
        this.longClientId = undefined;
        this.shortIds = new Map();      // long client id -> short id (client.ts:636-660)
        this.longIds = [];
        this.keyIds = new Map();        // property key -> id
        this.keys = [];
        this.valueIds = [];             // per key id: JSON(value) -> id (ids are per key: only equality matters)
        this.values = [];               // per key id: id -> value
        this.currentSeq = 0;
        this.minSeq = 0;
        this.msgQueue = [];
        this._delta = undefined;
        this._maintenance = undefined;
        this.expect = [];               // opArgs of the ops whose delta callback is still to come
        this.cbSegs = new WeakSet();    // the delta segments of the callbacks being delivered
    }

    get mergeTreeDeltaCallback() { return this._delta; }
    set mergeTreeDeltaCallback(cb) { this.engine._enableEvents(); this._delta = cb; }
    get mergeTreeMaintenanceCallback() { return this._maintenance; }
    set mergeTreeMaintenanceCallback(cb) { this.engine._enableEvents(); this._maintenance = cb; }

    _deliver(rows, lo, hi) {
        const cbs = [];
        for (let i = lo; i < hi; i++) {
            const o = EVREC * i;
            const op = rows.readInt8(o + 4), flags = rows.readUInt8(o + 5);
            if (flags & 1) cbs.push({ seq: rows.readInt32LE(o), operation: op, deltaSegments: [] });
            if (flags & 2) continue;  // a callback without delta segments
            const segment = { ordinal: rows.readInt32LE(o + 8), cachedLength: rows.readUInt32LE(o + 16) };
            if (op >= 0) {
                segment.position = rows.readInt32LE(o + 12);
                this.cbSegs.add(segment);  // getPosition answers with the position at callback time
            }
            const delta = { segment };
            if (op === ANNOTATE && !(flags & 4)) {  // (MT_EVF_NOPD: propertyDeltas undefined)
                const mask = rows.readUInt32LE(o + 20);
                delta.propertyDeltas = {};
                for (let k = 0; k < MAX_KEYS; k++) {
                    if (!((mask >>> k) & 1)) continue;
                    const v = rows.readUInt16LE(o + 24 + 2 * k);
                    delta.propertyDeltas[this.keys[k]] = v ? this.values[k][v] : null;
                }
            }
            cbs[cbs.length - 1].deltaSegments.push(delta);
        }
        for (const c of cbs) {
            if (c.operation >= 0) {
                const opArgs = this.expect.shift();
                if (this._delta) this._delta(opArgs, { operation: c.operation, deltaSegments: c.deltaSegments });
            } else if (this._maintenance) {
                // (sequenceNumber: the message being applied -- not in the reference's args)
                this._maintenance({ operation: c.operation, deltaSegments: c.deltaSegments, sequenceNumber: c.seq });
            }
        }
    }

    startOrUpdateCollaboration(longClientId, minSeq = 0, currentSeq = 0) {
        if (this.longClientId !== undefined) throw new Error("BatchClient: collaboration already started");
        this.longClientId = longClientId;
        this._shortId(longClientId);    // the observer is short id 0 (client.ts:1057-1062)
        this.currentSeq = currentSeq;
        this.minSeq = minSeq;
        if (minSeq || currentSeq) throw new Error("BatchClient: documents start empty at seq 0");
    }

    _shortId(longId) {
        let id = this.shortIds.get(longId);
        if (id === undefined) {
            // (short id 254 is NonCollabClient's, include/mtgpu.h: never a client's)
            if (this.longIds.length === NONCOLLAB_ID) this.longIds.push(undefined);
            id = this.longIds.length;
            if (id >= MAX_CLIENTS) throw new Error(`BatchClient: more than ${MAX_CLIENTS - 2} client ids in one document`);
            this.shortIds.set(longId, id);
            this.longIds.push(longId);
        }
        return id;
    }

    _pairs(props) {
        const out = [];
        for (const k of Object.keys(props || {})) {
            let kid = this.keyIds.get(k);
            if (kid === undefined) {
                kid = this.keys.length;
                if (kid >= MAX_KEYS) throw new Error(`BatchClient: more than ${MAX_KEYS} property keys`);
                this.keyIds.set(k, kid);
                this.keys.push(k);
                this.valueIds.push(new Map());
                this.values.push([undefined]);
                // the label keys whose block caches the engine tracks (mt_set_label_keys), declared
                // before the batch that carries the key's first op is submitted (BatchEngine._encode)
                if (k === "referenceTileLabels" || k === "referenceRangeLabels") {
                    this.engine.labelDecl.push([this.doc, k === "referenceTileLabels" ? kid : -1,
                        k === "referenceRangeLabels" ? kid : -1]);
                }
            }
            const v = props[k];
            let vid = 0;
            if (v !== null) {
                if (typeof v === "undefined" || typeof v === "function" || (typeof v === "number" && isNaN(v))) {
                    throw new Error("BatchClient: property values must be JSON values");
                }
                // objects and arrays (e.g. referenceTileLabels) are interned by content with sorted
                // keys: matchProperties compares them structurally (properties.ts:62-93)
                const key = canonicalJson(v);
                vid = this.valueIds[kid].get(key);
                if (vid === undefined) {
                    vid = this.values[kid].length;
                    if (vid > MAX_VALUES) throw new Error(`BatchClient: more than ${MAX_VALUES} values of property "${k}"`);
                    this.valueIds[kid].set(key, vid);
                    this.values[kid].push(v);
                }
            }
            out.push(kid, vid);
        }
        return out;
    }

    _record(msg, op, client, more) {
        const r = { seq: msg.sequenceNumber, ref: msg.referenceSequenceNumber, msn: msg.minimumSequenceNumber,
            client, type: NOOP, flags: more ? F_GROUP_MORE : 0, npairs: 0, pos1: 0, pos2: 0, payload: Buffer.alloc(0) };
        if (!op) return r;
        if (op.type === INSERT) {
            if (op.register || op.relativePos1) throw new Error("BatchClient: register/relative inserts unsupported");
            if (op.seg === "") return r;  // `if (op.seg)`: dropped before the tree (client.ts:403-407)
            let text, pairs = [];
            if (typeof op.seg === "string") text = op.seg;
            else if (op.seg && typeof op.seg === "object" && "text" in op.seg) {
                text = op.seg.text;
                if (op.seg.props) { r.flags |= F_PROPS; pairs = this._pairs(op.seg.props); }
            } else if (op.seg && typeof op.seg === "object" && "marker" in op.seg) {
                // Marker.fromJSONObject (mergeTree.ts:658-665): length 1, its ReferenceType as the one byte
                const rt = op.seg.marker.refType;
                if (!(Number.isInteger(rt) && rt >= 0 && rt <= 255)) throw new Error("BatchClient: marker refType out of range");
                text = String.fromCharCode(rt);
                r.flags |= F_MARKER;
                if (op.seg.props) { r.flags |= F_PROPS; pairs = this._pairs(op.seg.props); }
            } else throw new Error("BatchClient: only text and marker segments are supported");
            if (typeof text !== "string") throw new Error("BatchClient: segment text must be a string");
            // lengths and positions are UTF-16 code units (cachedLength = text.length, textSegment.ts:45):
            // Latin-1 bytes when every unit fits, else the wide form's 2 bytes per unit
            r.type = INSERT; r.pos1 = op.pos1;
            r.npairs = pairs.length / 2;
            r.text = text;
            r.pairs = pairs;
        } else if (op.type === REMOVE || op.type === ANNOTATE) {
            if (op.relativePos1 || op.relativePos2 || op.register) throw new Error("BatchClient: unsupported op form");
            r.type = op.type; r.pos1 = op.pos1; r.pos2 = op.pos2;
            if (op.type === ANNOTATE) {
                if (op.combiningOp) {
                    if (op.combiningOp.name !== "rewrite") throw new Error("BatchClient: combining ops unsupported");
                    r.flags |= F_REWRITE;
                }
                const pairs = this._pairs(op.props);
                r.npairs = pairs.length / 2;
                r.text = "";
                r.pairs = pairs;
            }
        } else {
            throw new Error(`BatchClient: op type ${op.type} unsupported`);
        }
        if (r.pairs) {  // the payload, narrow or wide (include/mtgpu.h MT_OP_WIDE)
            let wide = /[^\u0000-\u00ff]/.test(r.text);
            for (let q = 0; q < r.pairs.length; q += 2) wide = wide || r.pairs[q] >= NARROW_KEYS || r.pairs[q + 1] > 255;
            if (wide) {
                const pb = Buffer.alloc(3 * r.npairs);
                for (let q = 0; q < r.npairs; q++) {
                    pb.writeUInt8(r.pairs[2 * q], 3 * q);
                    pb.writeUInt16LE(r.pairs[2 * q + 1], 3 * q + 1);
                }
                r.type |= OP_WIDE;
                r.payload = Buffer.concat([Buffer.from(r.text, "utf16le"), pb]);
            } else {
                r.payload = Buffer.concat([Buffer.from(r.text, "latin1"), Buffer.from(r.pairs)]);
            }
            delete r.text;
            delete r.pairs;
        }
        return r;
    }

    // ---- an editing client (client.ts:163-214): local edits are queued as MT_SEQ_LOCAL records of
    // the client's own short id (0) and applied on the device in the local view; the client's own
    // sequenced messages, passed to applyMsg, are their acks (include/mtgpu.h)
    _local(op) {
        if (this.longClientId === undefined) throw new Error("BatchClient: startOrUpdateCollaboration first");
        const msg = { sequenceNumber: -1, referenceSequenceNumber: this.currentSeq, minimumSequenceNumber: 0 };
        const r = this._record(msg, op, this._shortId(this.longClientId), false);
        if (r.type === NOOP) return undefined;  // insertSegmentLocal: nothing for an empty segment
        if ((r.type & OP_WIDE) || r.client >= NARROW_CLIENTS) {
            throw new Error("BatchClient: an editing client's document stays within the narrow limits (include/mtgpu.h)");
        }
        this.queue.push(r);
        if (this.engine.recording) this.expect.push({ op });  // a local edit's callback: no sequencedMessage
        this.engine.pending += 1;
        if (this.engine._syncPoint) this.engine._syncPoint(this);  // (a host-only stub engine has none)
        return op;
    }
    /** TestClient.insertTextLocal (testClient.ts:133-143) -> insertSegmentLocal: the insert op. */
    insertTextLocal(pos, text, props) {
        return this._local({ type: INSERT, pos1: pos, seg: props ? { text, props } : text });
    }
    /** TestClient.insertMarkerLocal (testClient.ts:178-188). */
    insertMarkerLocal(pos, refType, props) {
        const seg = { marker: { refType } };
        if (props) seg.props = props;
        return this._local({ type: INSERT, pos1: pos, seg });
    }
    /**
     * Client.regeneratePendingOp (client.ts:855-893) on reconnect, for the oldest pending edit, whose
     * op is `resetOp` (the segment group is implied: the head of the pending queue): the new op to
     * resubmit -- one op per segment, a GROUP op when there are several (or none).
     */
    regeneratePendingOp(resetOp) {
        const members = resetOp.type === GROUP ? resetOp.ops : [resetOp];
        for (const m of members) {
            const msg = { sequenceNumber: -2, referenceSequenceNumber: this.currentSeq, minimumSequenceNumber: 0 };
            const r = this._record(msg, m, this._shortId(this.longClientId), false);
            if (r.type === NOOP) throw new Error("BatchClient: nothing to regenerate");
            this.queue.push(r);
            this.engine.pending += 1;
        }
        this.engine.flush();
        this._checkError();
        const [recs, pay] = native.regenDrain(this.engine.handle, this.doc);
        const ops = [];
        for (let o = 0; o + REC <= recs.length && recs.length >= REC; o += REC) {
            const type = recs.readUInt8(o + 14), flags = recs.readUInt8(o + 15);
            if (type === NOOP) continue;  // one header per regenerated op
            const pos1 = recs.readInt32LE(o + 16), pos2 = recs.readInt32LE(o + 20);
            const off = recs.readUInt32LE(o + 24), len = recs.readUInt32LE(o + 28);
            const np = (flags >> 3) & 15;
            const props = {};
            for (let q = 0; q < np; q++) {
                const k = pay.readUInt8(off + len - 2 * np + 2 * q), v = pay.readUInt8(off + len - 2 * np + 2 * q + 1);
                props[this.keys[k]] = v ? this.values[k][v] : null;
            }
            if (type === INSERT) {
                const text = pay.toString("latin1", off, off + len - 2 * np);
                let seg;
                if (flags & F_MARKER) seg = { marker: { refType: text.charCodeAt(0) } };
                else seg = (flags & F_PROPS) ? { text } : text;
                if (flags & F_PROPS) seg.props = props;
                ops.push({ type: INSERT, pos1, seg });
            } else if (type === REMOVE) {
                ops.push({ type: REMOVE, pos1, pos2 });
            } else {
                const op = { type: ANNOTATE, pos1, pos2, props };
                if (flags & F_REWRITE) op.combiningOp = { name: "rewrite" };
                ops.push(op);
            }
        }
        return ops.length === 1 ? ops[0] : { type: GROUP, ops };
    }

    /** Client.removeRangeLocal (client.ts:188-195). */
    removeRangeLocal(start, end) { return this._local({ type: REMOVE, pos1: start, pos2: end }); }
    /** Client.annotateRangeLocal (client.ts:163-179). */
    annotateRangeLocal(start, end, props, combiningOp) {
        const op = { type: ANNOTATE, pos1: start, pos2: end, props };
        if (combiningOp) op.combiningOp = combiningOp;
        return this._local(op);
    }

    /** Client.applyMsg (client.ts:797-819): queued, applied in the next device batch.  A message of
     * this client's own long id acks its oldest pending local edit (client.ts:804-806). */
    applyMsg(msg) {
        const client = this._shortId(msg.clientId);
        const ack = msg.type === "op" && msg.clientId === this.longClientId;  // fires no delta callback
        const op = msg.type === "op" ? msg.contents : undefined;
        const members = op && op.type === GROUP ? op.ops : [op];
        members.forEach((m, i) => {
            const r = this._record(msg, m, client, i + 1 < members.length);
            this.queue.push(r);
            // every applied op fires one delta callback; an empty-string insert is dropped before
            // the tree (client.ts:403-407), a non-op message has none
            if (this.engine.recording && r.type !== NOOP && !ack) {
                this.expect.push({ op: m, groupOp: op.type === GROUP ? op : undefined, sequencedMessage: msg });
            }
            this.engine.pending += 1;
            // (syncCallbacks: each member applied and its callback delivered in turn, as the reference
            // fires one callback per member inside the GROUP's apply)
            if (this.engine._syncPoint) this.engine._syncPoint(this);  // (a host-only stub engine has none)
        });
        // (after the members, as updateSeqNumbers follows the op: client.ts:818; a listener reading
        // getCurrentSeq() inside the callback sees the previous one, as the reference's does)
        this.currentSeq = msg.sequenceNumber;
        this.minSeq = Math.max(this.minSeq, msg.minimumSequenceNumber);
    }

    _checkError() {
        const [code, seq] = native.docError(this.engine.handle, this.doc);
        if (code) {
            const msgs = { 1: "Incoming remote op sequence# <= local collabWindow's currentSequence#",
                2: "Incoming remote op minSequence# < local collabWindow's minSequence#", 3: "MergeTree insert failed",
                4: "device capacity exceeded", 5: "text arena exhausted", 6: "id limits exceeded", 7: "malformed op" };
            throw new Error(`${msgs[code] || code} (seq ${seq})`);
        }
    }

    getText() { this.engine.flush(); this._checkError(); return native.getText(this.engine.handle, this.doc); }

    /**
     * Client.findTile (client.ts:1073-1076): the tile holding `tileLabel` in its
     * "referenceTileLabels" property nearest to startPos -- at or before it (preceding), else at or
     * after it -- as {tile: {ordinal}, pos}, or undefined (include/mtgpu.h "findTile").
     */
    findTile(startPos, tileLabel, preceding = true) {
        this.engine.flush();
        this._checkError();
        const q = Buffer.alloc(48);
        this._labelQuery(q, 0, "referenceTileLabels", startPos, tileLabel, preceding);
        const r = native.findTiles(this.engine.handle, q);
        const pos = r.readInt32LE(0);
        return pos < 0 ? undefined : { tile: { ordinal: r.readInt32LE(4) }, pos };
    }
    // one 48-byte mt_tile_query: `label` as the set of value ids whose label arrays (property `key`) hold it
    _labelQuery(q, off, key, pos, label, preceding) {
        q.writeUInt32LE(this.doc, off);
        q.writeInt32LE(pos, off + 4);
        const kid = this.keyIds.get(key);
        q.writeUInt8(kid === undefined ? 0xff : kid, off + 8);
        q.writeUInt8(preceding ? 1 : 0, off + 9);
        const vals = kid === undefined ? [undefined] : this.values[kid];
        // (the query's label mask covers value ids below 256 of the label key)
        if (vals.length > 256) throw new Error(`BatchClient: more than 255 values of "${key}" for a label query`);
        for (let v = 1; v < vals.length; v++) {
            const labels = vals[v];
            if (Array.isArray(labels) && labels.includes(label)) {
                const o = off + 12 + 4 * (v >> 5);
                q.writeUInt32LE((q.readUInt32LE(o) | (1 << (v & 31))) >>> 0, o);
            }
        }
    }

    /**
     * Client.getStackContext (client.ts:946-948): for each of `rangeLabels` that a live NestBegin /
     * NestEnd marker at or before startPos carries in "referenceRangeLabels", the stack
     * applyRangeReference folds them into, as {items: [{ordinal, pos, refType}, ...]} bottom to top
     * (include/mtgpu.h "range stacks").
     */
    getStackContext(startPos, rangeLabels) {
        this.engine.flush();
        this._checkError();
        const n = rangeLabels.length;
        const q = Buffer.alloc(48 * n);
        rangeLabels.forEach((l, i) => this._labelQuery(q, 48 * i, "referenceRangeLabels", startPos, l, false));
        let cap = 16;
        let [items, depth] = native.rangeStacks(this.engine.handle, q, cap);
        let deepest = 0;
        for (let i = 0; i < n; i++) deepest = Math.max(deepest, depth.readUInt32LE(4 * i) & 0x7fffffff);
        if (deepest > cap) {
            cap = deepest;
            [items, depth] = native.rangeStacks(this.engine.handle, q, cap);
        }
        const stacks = {};
        rangeLabels.forEach((l, i) => {
            const w = depth.readUInt32LE(4 * i);
            if (!(w & 0x80000000)) return;  // no marker of the label: absent, as in the reference's map
            const st = [];
            for (let k = 0; k < (w & 0x7fffffff); k++) {
                const o = 12 * (i * cap + k);
                st.push({ pos: items.readInt32LE(o), ordinal: items.readInt32LE(o + 4), refType: items.readUInt32LE(o + 8) });
            }
            stacks[l] = { items: st };
        });
        return stacks;
    }

    getLength() { this.engine.flush(); this._checkError(); return native.getLength(this.engine.handle, this.doc); }
    getCurrentSeq() { return this.currentSeq; }
    getClientId() { return 0; }
    getLongClientId(id) { return this.longIds[id]; }

    /** Canonical state with long client ids and original property keys/values. */
    getState() {
        this.engine.flush();
        const st = JSON.parse(native.getState(this.engine.handle, this.doc));
        for (const s of st.segs) {
            s[2] = s[2] < 0 ? s[2] : this.longIds[s[2]];  // (-2: NonCollabClient, a segment loaded below the MSN)
            if (s[4] !== -1) s[4] = this.longIds[s[4]];
            s[5] = s[5].map((x) => this.longIds[x]);
            if (s[6]) {
                const p = {};
                for (const k of Object.keys(s[6])) {
                    const kid = parseInt(k.slice(1), 10);
                    p[this.keys[kid]] = this.values[kid][s[6][k]];
                }
                s[6] = p;
            }
        }
        return st;
    }

    // ---- the read surface over the applied state (client.ts:275-311, 838-847, 1004-1040) --------
    // A segment is a plain descriptor of the state it was read from -- {ordinal, position (local
    // view), cachedLength, seq, clientId, removedSeq, removedClientId (short ids), properties,
    // text | refType} -- named by its ordinal (its index among the document's linked segments): the
    // device keeps no segment objects, so a descriptor is valid until the document next changes.
    _segments() {
        const st = this.getState();
        let pos = 0;
        return st.segs.map((s, i) => {
            const marker = s[0] !== null && typeof s[0] === "object";
            const len = marker ? 1 : s[0].length;
            const removed = s[4] !== -1;
            const d = { ordinal: i, position: pos, cachedLength: len, seq: s[1],
                clientId: typeof s[2] === "string" ? this._shortId(s[2]) : s[2],
                removedSeq: removed ? s[3] : undefined, removedClientId: removed ? this._shortId(s[4]) : undefined,
                removedClientOverlap: s[5].length ? s[5].map((x) => this._shortId(x)) : undefined,
                properties: s[6] || undefined };
            if (marker) d.refType = s[0].marker; else d.text = s[0];
            if (!removed) pos += len;
            return d;
        });
    }
    // nodeLength of a leaf (mergeTree.ts:1659-1697): the local view (localNetLength) or a remote
    // client's view at refSeq
    static _viewLength(d, refSeq, clientId, local) {
        const removed = d.removedSeq !== undefined;
        if (local) return removed ? 0 : d.cachedLength;
        if (!(d.clientId === clientId || (d.seq !== -1 && d.seq <= refSeq))) return 0;
        if (removed && (d.removedClientId === clientId || (d.removedClientOverlap || []).includes(clientId) ||
            (d.removedSeq !== -1 && d.removedSeq <= refSeq))) return 0;
        return d.cachedLength;
    }
    // ---- device queries (include/mtgpu.h mt_resolve_positions / mt_segment_infos): one wave per
    // query over the document's state in HBM, no whole-document read.  A descriptor from them carries
    // {ordinal, position, cachedLength} at once; its other fields are read from the device on first
    // access (one segment's row), so it too is valid until the document next changes.
    _resolve(kind, pos, refSeq, clientId) {
        this.engine.flush();
        this._checkError();
        const q = Buffer.alloc(16);
        q.writeUInt32LE(this.doc, 0);
        q.writeInt32LE(pos, 4);
        q.writeInt32LE(refSeq === undefined ? POS_LOCAL : refSeq, 8);
        q.writeUInt16LE(clientId || 0, 12);
        q.writeUInt16LE(kind, 14);
        const r = native.resolvePositions(this.engine.handle, q);
        return { ordinal: r.readInt32LE(0), offset: r.readInt32LE(4), position: r.readInt32LE(8), length: r.readUInt32LE(12) };
    }
    _descriptor(ordinal, position, cachedLength) {
        // the segment's fields are gathered now (one small device gather), so the descriptor is a
        // self-consistent snapshot of the segment as of this query; its text is read on first access,
        // which must come before the document next changes (the arena is rewritten by later ops)
        const self = this, gen = this.engine.gen;
        const docs = Buffer.alloc(4), ords = Buffer.alloc(4);
        docs.writeUInt32LE(self.doc, 0);
        ords.writeInt32LE(ordinal, 0);
        const b = native.segmentInfos(self.engine.handle, docs, ords);
        const flags = b.readUInt32LE(20), removed = (flags & 1) !== 0;
        const overlap = [];
        const lo = b.readUInt32LE(32), hi = b.readUInt32LE(36);
        for (let c = 0; c < 32; c++) if ((lo >>> c) & 1) overlap.push(c);
        for (let c = 0; c < 32; c++) if ((hi >>> c) & 1) overlap.push(32 + c);
        for (let q = 0; q < OVX_IDS; q++) { const c = b.readUInt16LE(104 + 2 * q); if (!c) break; overlap.push(c); }
        let properties;
        if (flags & 2) {
            properties = {};
            for (let kid = 0; kid < MAX_KEYS; kid++) {
                const vid = b.readUInt16LE(40 + 2 * kid);
                if (vid) properties[self.keys[kid]] = self.values[kid][vid];
            }
        }
        const marker = (flags & 16) !== 0, toff = b.readUInt32LE(24), len = b.readUInt32LE(16);
        let txt;
        const text = () => {
            if (txt === undefined) {
                if (self.engine.gen !== gen || self.engine.pending) {
                    throw new Error("BatchClient: a segment's text read after the document changed (query it again)");
                }
                txt = native.segmentText(self.engine.handle, self.doc, toff, len);
            }
            return txt;
        };
        const d = { ordinal, position, cachedLength, seq: b.readInt32LE(0), clientId: b.readInt32LE(8),
            removedSeq: removed ? b.readInt32LE(4) : undefined, removedClientId: removed ? b.readInt32LE(12) : undefined,
            removedClientOverlap: overlap.length ? overlap : undefined, properties };
        Object.defineProperty(d, "text", { get: () => (marker ? undefined : text()), enumerable: true });
        Object.defineProperty(d, "refType", { get: () => (marker ? text().charCodeAt(0) : undefined), enumerable: true });
        return d;
    }
    /** Client.getContainingSegment (client.ts:1004-1007): {segment, offset} in the local view. */
    getContainingSegment(pos) {
        const r = this._resolve(POS_CONTAINING, pos);
        if (r.ordinal < 0) return { segment: undefined, offset: undefined };
        return { segment: this._descriptor(r.ordinal, r.position, r.length), offset: r.offset };
    }
    /** Client.getPropertiesAtPosition (client.ts:1009-1023). */
    getPropertiesAtPosition(pos) {
        const seg = this.getContainingSegment(pos).segment;
        return seg ? seg.properties : undefined;
    }
    /** Client.getRangeExtentsOfPosition (client.ts:1024-1040). */
    getRangeExtentsOfPosition(pos) {
        const r = this._resolve(POS_CONTAINING, pos);
        return r.ordinal >= 0 ? { posStart: r.position, posAfterEnd: r.position + r.length }
            : { posStart: undefined, posAfterEnd: undefined };
    }
    /** Client.getPosition (client.ts:290-292): the local-view position of the segment (by ordinal). */
    getPosition(segment) {
        // a delta segment of the callback being delivered: its position at callback time (the reference's
        // getPosition inside the listener; the ordinal may have moved since, e.g. by zamboni)
        if (this.cbSegs.has(segment)) return segment.position;
        const r = this._resolve(POS_OF_ORDINAL, segment.ordinal);
        return r.ordinal >= 0 ? r.position : 0;
    }
    /**
     * Client.walkSegments (client.ts:275-284, MergeTree.mapRange / nodeMap mergeTree.ts:2903-2960):
     * handler(segment, pos, refSeq, clientId, start, end, accum) for every segment of the local view
     * overlapping [start, end) (start / end relative to the segment), until it returns a falsy value.
     * splitRange (which splits segments in place) is not supported.
     */
    walkSegments(handler, start, end, accum, splitRange = false) {
        if (splitRange) throw new Error("BatchClient.walkSegments: splitRange is not supported");
        const segs = this._segments();
        if (start === undefined) start = 0;
        if (end === undefined) end = segs.reduce((a, d) => a + (d.removedSeq === undefined ? d.cachedLength : 0), 0);
        let pos = 0;
        for (const d of segs) {
            const len = d.removedSeq === undefined ? d.cachedLength : 0;
            if (end > 0 && len > 0 && start < len && !handler(d, pos, this.currentSeq, this.getClientId(), start, end, accum)) {
                break;
            }
            pos += len;
            start -= len;
            end -= len;
        }
    }
    /**
     * Client.getMarkerFromId (client.ts:311-313): the marker whose "markerId" property is id.  The
     * reference's id map keeps markers after their removal; here a removed marker is found while it
     * is still in the document (until zamboni unlinks it), a live one first.
     */
    getMarkerFromId(id) {
        let found;
        for (const d of this._segments()) {
            if (d.refType !== undefined && d.properties && d.properties.markerId === id &&
                (found === undefined || d.removedSeq === undefined || found.removedSeq !== undefined)) {
                found = d;
            }
        }
        return found;
    }
    /**
     * Client.resolveRemoteClientPosition (client.ts:838-847, mergeTree.ts:2105-2127): a remote
     * client's position at its refSeq, as a local position (undefined past its length).
     */
    resolveRemoteClientPosition(remoteClientPosition, remoteClientRefSeq, remoteClientId) {
        const cid = this._shortId(remoteClientId);
        const local = cid === this._shortId(this.longClientId);  // (nodeLength: the own client sees the local view)
        const r = this._resolve(POS_CONTAINING, remoteClientPosition, local ? undefined : remoteClientRefSeq, cid);
        if (r.ordinal >= 0) return r.position + r.offset;
        if (r.offset === 0) return r.position;  // at the end of the remote view: the local length
        return undefined;
    }

    // ---- TestClient helpers (src/test/testClient.ts:112-234) --------------------------------
    makeOpMessage(op, seq = -1, refSeq = this.currentSeq, longClientId, minSeqNumber = 0) {
        return { clientId: longClientId === undefined ? this.longClientId : longClientId, clientSequenceNumber: 1,
            contents: op, metadata: undefined, minimumSequenceNumber: minSeqNumber, origin: null,
            referenceSequenceNumber: refSeq, sequenceNumber: seq, timestamp: Date.now(), term: 1, traces: [],
            type: "op" };
    }
    insertTextRemote(pos, text, props, seq, refSeq, longClientId) {
        const seg = props ? { text, props } : text;
        this.applyMsg(this.makeOpMessage({ type: INSERT, pos1: pos, seg }, seq, refSeq, longClientId));
    }
    /** TestClient.insertMarkerRemote (testClient.ts:190-207). */
    insertMarkerRemote(pos, markerDef, props, seq, refSeq, longClientId) {
        const seg = { marker: { refType: markerDef.refType } };
        if (props) seg.props = props;
        this.applyMsg(this.makeOpMessage({ type: INSERT, pos1: pos, seg }, seq, refSeq, longClientId));
    }
    removeRangeRemote(start, end, seq, refSeq, longClientId) {
        this.applyMsg(this.makeOpMessage({ type: REMOVE, pos1: start, pos2: end }, seq, refSeq, longClientId));
    }
    enqueueMsg(msg) { this.msgQueue.push(msg); }
    dequeueMsg() { return this.msgQueue.shift(); }
    getMessageCount() { return this.msgQueue.length; }
    applyMessages(msgCount) {
        for (let n = msgCount; n > 0; n--) {
            const m = this.msgQueue.shift();
            if (!m) break;
            this.applyMsg(m);
        }
        return true;
    }
}

module.exports = { BatchEngine, BatchClient, native };
