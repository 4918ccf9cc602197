"use strict";
// sequenceDeltaEvent.js -- SequenceDeltaEvent / SequenceMaintenanceEvent
// (packages/dds/sequence/src/sequenceDeltaEvent.ts:26-161) over the device engine's delta callbacks, and
// the event side of SharedSegmentSequence (sequence.ts:131-149): a BatchClient whose "sequenceDelta" /
// "maintenance" listeners get one event object per merge-tree callback.
//
//   const { SequenceEvents } = require("./sequenceDeltaEvent.js");
//   const seq = new SequenceEvents(client);          // client: a BatchClient
//   seq.on("sequenceDelta", (event, target) => { event.ranges; event.first; event.isLocal; ... });
//
// The engine records the callbacks during the batch and BatchClient delivers them, in firing order,
// after it (include/mtgpu.h "delta / maintenance events"); each event is built then.  A delta
// segment is {ordinal, position, cachedLength} as of the callback (include/mtgpu.h): ranges[i].position
// is that callback-time position -- the "point in time state at the time the operation was applied"
// the reference documents (sequenceDeltaEvent.ts:19-25); the reference computes it lazily with
// client.getPosition(segment) (:41-52), which equals it when read inside the listener.  Ranges are
// sorted by ordinal (SortedSegmentSet, sortedSegmentSet.ts), which is document order.  Maintenance
// callbacks carry no position (maintenance delta segments may be unlinked, :48).
const { EventEmitter } = require("events");

class SequenceEvent {
    constructor(deltaArgs, client) {
        this.deltaArgs = deltaArgs;
        this.deltaOperation = deltaArgs.operation;
        this.isEmpty = deltaArgs.deltaSegments.length === 0;
        this._client = client;
        this._ranges = undefined;
    }

    /** The in-order ranges affected by this delta (not necessarily continuous). */
    get ranges() {
        if (this._ranges === undefined) {
            const byOrdinal = new Map();  // SortedSegmentSet.addOrUpdate: one range per segment
            for (const d of this.deltaArgs.deltaSegments) {
                if (!byOrdinal.has(d.segment.ordinal)) {
                    byOrdinal.set(d.segment.ordinal, { operation: this.deltaArgs.operation, position: d.segment.position,
                        propertyDeltas: d.propertyDeltas, segment: d.segment });
                }
            }
            this._ranges = Array.from(byOrdinal.values()).sort((a, b) => a.segment.ordinal - b.segment.ordinal);
        }
        return this._ranges;
    }

    /** The client id of the client the events are delivered to (mergeTreeClient.longClientId). */
    get clientId() { return this._client.longClientId; }
    get first() { return this.isEmpty ? undefined : this.ranges[0]; }
    get last() { return this.isEmpty ? undefined : this.ranges[this.ranges.length - 1]; }
}

/** The event of "sequenceDelta" listeners: one per op callback (a GROUP op: one per member). */
class SequenceDeltaEvent extends SequenceEvent {
    constructor(opArgs, deltaArgs, client) {
        super(deltaArgs, client);
        this.opArgs = opArgs;
        this.isLocal = opArgs.sequencedMessage === undefined;
    }
}

/** The event of "maintenance" listeners (APPEND / SPLIT / UNLINK). */
class SequenceMaintenanceEvent extends SequenceEvent {}

/**
 * SharedSegmentSequence's event surface (sequence.ts:131-149) for one BatchClient: the first
 * "sequenceDelta" (or "maintenance") listener installs the client's merge-tree callback, which wraps
 * each callback in an event; removing the last listener uninstalls it.
 */
class SequenceEvents extends EventEmitter {
    constructor(client) {
        super();
        this.client = client;
        this.on("newListener", (event) => {
            if (event === "sequenceDelta" && !this.client.mergeTreeDeltaCallback) {
                this.client.mergeTreeDeltaCallback = (opArgs, deltaArgs) => {
                    this.emit("sequenceDelta", new SequenceDeltaEvent(opArgs, deltaArgs, this.client), this);
                };
            } else if (event === "maintenance" && !this.client.mergeTreeMaintenanceCallback) {
                this.client.mergeTreeMaintenanceCallback = (args) => {
                    this.emit("maintenance", new SequenceMaintenanceEvent(args, this.client), this);
                };
            }
        });
        this.on("removeListener", (event) => {
            if (event === "sequenceDelta" && this.listenerCount(event) === 0) this.client.mergeTreeDeltaCallback = undefined;
            if (event === "maintenance" && this.listenerCount(event) === 0) this.client.mergeTreeMaintenanceCallback = undefined;
        });
    }
}

module.exports = { SequenceDeltaEvent, SequenceMaintenanceEvent, SequenceEvent, SequenceEvents };
