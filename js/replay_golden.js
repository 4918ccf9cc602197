"use strict";
// Replays an MTLOG through BatchClient (one observer per document, all documents on one
// BatchEngine) and prints one JSON line per document: {doc, state (long ids), text}.
const { BatchEngine } = require("./batchClient.js");
const { loadLog, messages } = require("./mtlog.js");

const log = loadLog(process.argv[2]);
const opsPerLaunch = parseInt(process.argv[3] || "0", 10);
const eng = new BatchEngine({ maxDocs: log.nDocs, opsPerLaunch });
const clients = [];
for (let d = 0; d < log.nDocs; d++) {
    const c = eng.createClient();
    c.startOrUpdateCollaboration("observer");
    for (const m of messages(log, d)) c.applyMsg(m);
    clients.push(c);
}
const out = [];
for (let d = 0; d < log.nDocs; d++) {
    const c = clients[d];
    out.push(JSON.stringify({ doc: d, text: c.getText(), length: c.getLength(), state: c.getState() }));
}
process.stdout.write(out.join("\n") + "\n");
