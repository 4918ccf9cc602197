"use strict";
// Replays an MTLOG through BatchClient (one observer per document, all documents on one
// BatchEngine) and prints one JSON line per document: {doc, state (long ids), text}.
//   node replay_golden.js <log> [opsPerLaunch] [events]
// "events": mergeTreeDeltaCallback / mergeTreeMaintenanceCallback set on every client, a flush
// every 40 messages, and each line also carries the callbacks in the canonical event form of
// fluidframework_amd/events.py ([seq, operation, [[ordinal, position, cachedLength, propertyDeltas]]]).
const { BatchEngine } = require("./batchClient.js");
const { loadLog, messages } = require("./mtlog.js");

const log = loadLog(process.argv[2]);
const opsPerLaunch = parseInt(process.argv[3] || "0", 10);
const withEvents = process.argv[4] === "events";
const eng = new BatchEngine({ maxDocs: log.nDocs, opsPerLaunch });
const clients = [], events = [];
for (let d = 0; d < log.nDocs; d++) {
    const c = eng.createClient();
    c.startOrUpdateCollaboration("observer");
    const ev = [];
    events.push(ev);
    if (withEvents) {
        const seg = (x, pd) => [x.segment.ordinal, x.segment.position === undefined ? -1 : x.segment.position,
            x.segment.cachedLength, pd];
        c.mergeTreeDeltaCallback = (opArgs, args) => ev.push([opArgs.sequencedMessage.sequenceNumber, args.operation,
            args.deltaSegments.map((x) => seg(x, args.operation === 2 ? sortKeys(x.propertyDeltas) : null))]);
        c.mergeTreeMaintenanceCallback = (args) => ev.push([args.sequenceNumber, args.operation,
            args.deltaSegments.map((x) => seg(x, null))]);
    }
    let n = 0;
    for (const m of messages(log, d)) {
        c.applyMsg(m);
        if (withEvents && ++n % 40 === 0) eng.flush();
    }
    clients.push(c);
}

function sortKeys(pd) {
    const o = {};
    for (const k of Object.keys(pd).sort((a, b) => parseInt(a.slice(1), 10) - parseInt(b.slice(1), 10))) o[k] = pd[k];
    return o;
}

const out = [];
for (let d = 0; d < log.nDocs; d++) {
    const c = clients[d];
    let text = null, length = null, err = null;
    try {
        text = c.getText();
        length = c.getLength();
    } catch (e) {
        err = String(e.message || e);
    }
    const line = { doc: d, text, length, err, state: c.getState() };
    if (withEvents) line.events = events[d];
    out.push(JSON.stringify(line));
}
process.stdout.write(out.join("\n") + "\n");
