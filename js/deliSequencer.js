"use strict";
// deliSequencer.js -- the ordering service's per-document sequencer over the MI355X engine
// (CommonJS, node 12).
//
// DeliSequencer replaces a DeliLambda per document (server/routerlicious/packages/lambdas/src/
// deli/lambda.ts:87-171) for many documents at once: queue(doc, rawMessage) takes an
// IRawOperationMessage (clientId, operation {type, clientSequenceNumber,
// referenceSequenceNumber, contents, data}); flush() tickets every queued message on the GPU
// (DeliLambda.ticket, lambda.ts:255-544) and returns, per message in queue order, what the
// lambda would have produced: a sequenced message (sequenceNumber, minimumSequenceNumber,
// referenceSequenceNumber) and whether it is sent now / later / never, a nack with its reason,
// or nothing (a dropped duplicate).  Client ids are interned per document (short ids < 512: include/
// mtgpu.h MT_DELI_MAX_CLIENTS; past 63 the document is ticketed by the engine's wide form).
const path = require("path");

const native = require(path.join(__dirname, "mtgpu.node"));

const OP = 0, NOOP = 1, NOOP_DATA = 2, JOIN = 3, LEAVE = 4, SERVER_NOOP = 5, NOCLIENT = 6, CONTROL = 7;
const STATUS = ["dropped", "sent", "later", "never", "nack", "nack", "nack", "halted"];
const NACK_REASON = { 4: "Gap detected in incoming op", 5: "Nonexistent client", 6: "Refseq below msn" };
const MAX_CLIENTS = 512;  // include/mtgpu.h MT_DELI_MAX_CLIENTS
const REC = 16;

class DeliSequencer {
    constructor(opts = {}) {
        this.maxDocs = opts.maxDocs || 1;
        this.handle = native.createDeli({ device: opts.device || 0, maxDocs: this.maxDocs });
        this.ids = Array.from({ length: this.maxDocs }, () => new Map());  // long client id -> short
        // short ids given back by processed leaves, reused before new ones (Fluid gives every
        // connection a new client id, so a long-lived document sees far more than 512 of them)
        this.free = Array.from({ length: this.maxDocs }, () => []);
        this.next = new Uint32Array(this.maxDocs);
        this.queues = Array.from({ length: this.maxDocs }, () => []);
        this.pending = 0;
    }

    _short(doc, longId) {
        const m = this.ids[doc];
        let s = m.get(longId);
        if (s === undefined) {
            s = this._freeSlot(doc, true);
            m.set(longId, s);
        }
        return s;
    }

    // a short id no long id holds: its device record is not joined (never used, or cleared by the
    // leave that gave it back).  take = reserve it for a new long id.
    _freeSlot(doc, take) {
        const f = this.free[doc];
        if (f.length) return take ? f.shift() : f[0];
        const s = this.next[doc];
        if (s >= MAX_CLIENTS) {
            throw new Error(`deli: more than ${MAX_CLIENTS} concurrently known clients in document ${doc}`);
        }
        if (take) this.next[doc] = s + 1;
        return s;
    }

    // IRawOperationMessage -> [kind, short client, csn, refSeq] (lambda.ts:263, 280-306, 414-443)
    _encode(doc, msg) {
        const op = msg.operation;
        const csn = op.clientSequenceNumber === undefined ? -1 : op.clientSequenceNumber;
        const ref = op.referenceSequenceNumber === undefined ? -1 : op.referenceSequenceNumber;
        if (msg.clientId) {
            const kind = op.type === "noop" ? (op.contents === null ? NOOP : NOOP_DATA) : OP;
            return [kind, this._short(doc, msg.clientId), csn, ref];
        }
        switch (op.type) {
            case "join": return [JOIN, this._short(doc, JSON.parse(op.data).clientId), csn, ref];
            case "leave": {
                // a leave of a client this document never saw is dropped by ticket() (lambda.ts:281-285):
                // it takes any unjoined slot and interns nothing
                const leaver = JSON.parse(op.data);
                const s = this.ids[doc].get(leaver);
                return [LEAVE, s === undefined ? this._freeSlot(doc, false) : s, csn, ref, leaver];
            }
            case "noop": return [SERVER_NOOP, 0, csn, ref];
            case "noClient": return [NOCLIENT, 0, csn, ref];
            case "control": return [CONTROL, 0, csn, ref];
            default: throw new Error(`deli: unsupported system message type ${op.type}`);
        }
    }

    queue(doc, rawMessage) {
        if (doc < 0 || doc >= this.maxDocs) throw new RangeError(`document ${doc}`);
        this.queues[doc].push([rawMessage, this._encode(doc, rawMessage)]);
        this.pending++;
    }

    // Ticket every queued message (one GPU launch); returns per document the outputs in order.
    flush() {
        const n = this.pending;
        const msgs = Buffer.alloc(Math.max(1, n) * REC);
        const rowPtr = new Uint32Array(this.maxDocs + 1);
        let k = 0;
        for (let d = 0; d < this.maxDocs; d++) {
            rowPtr[d] = k;
            for (const [, [kind, c, csn, ref]] of this.queues[d]) {
                const o = k * REC;
                msgs.writeInt32LE(csn, o);
                msgs.writeInt32LE(ref, o + 4);
                msgs.writeUInt16LE(c, o + 8);
                msgs.writeUInt8(kind, o + 10);
                k++;
            }
        }
        rowPtr[this.maxDocs] = k;
        const t = native.deliTicket(this.handle, msgs.subarray(0, n * REC), rowPtr);
        const out = [];
        k = 0;
        for (let d = 0; d < this.maxDocs; d++) {
            const res = [];
            for (const [raw, enc] of this.queues[d]) {
                const o = k * REC;
                const status = t.readUInt8(o + 12);
                if (enc[0] === LEAVE && enc[4] !== undefined && this.ids[d].get(enc[4]) === enc[1] &&
                    status !== 7) {
                    // after its leave the client is out of the ClientSequenceNumberManager
                    // (removeClient, lambda.ts:281-285): its short id is free again
                    this.ids[d].delete(enc[4]);
                    this.free[d].push(enc[1]);
                }
                const r = { status: STATUS[status], message: raw };
                if (status === 1 || status === 2 || status === 3) {
                    r.sequenceNumber = t.readInt32LE(o);
                    r.minimumSequenceNumber = t.readInt32LE(o + 4);
                    r.referenceSequenceNumber = t.readInt32LE(o + 8);
                } else if (status >= 4 && status <= 6) {
                    r.nack = { reason: NACK_REASON[status], sequenceNumber: t.readInt32LE(o) };
                }
                res.push(r);
                k++;
            }
            out.push(res);
            this.queues[d] = [];
        }
        this.pending = 0;
        return out;
    }

    error(doc) {
        return native.deliError(this.handle, doc);
    }
}

module.exports = { DeliSequencer, OP, NOOP, NOOP_DATA, JOIN, LEAVE, SERVER_NOOP, NOCLIENT, CONTROL };
