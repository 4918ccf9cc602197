"use strict";
// getStackContext through the Node surface: the tiles_* logs replayed into BatchClients (range labels
// on property key <rangeKey> as "referenceRangeLabels" arrays, js/mtlog.js), then every query of the
// reference's fixture asked with BatchClient.getStackContext; one JSON line per document {doc, answers}.
//   node replay_stacks.js <log.mtlog> <stacks.expected.jsonl> <logName> [rangeKey]
const fs = require("fs");
const { BatchEngine } = require("./batchClient.js");
const { loadLog, messages } = require("./mtlog.js");

const log = loadLog(process.argv[2]);
const rows = fs.readFileSync(process.argv[3], "utf8").split("\n").filter((x) => x.trim()).map((x) => JSON.parse(x))
    .filter((r) => r.log === process.argv[4]);
const rangeKey = parseInt(process.argv[5] || "1", 10);
const eng = new BatchEngine({ maxDocs: log.nDocs, opsPerLaunch: 32 });
const clients = [];
for (let d = 0; d < log.nDocs; d++) {
    const c = eng.createClient();
    c.startOrUpdateCollaboration("observer");
    for (const m of messages(log, d, { rangeKey })) c.applyMsg(m);
    clients.push(c);
}
const out = rows.map((r) => JSON.stringify({ doc: r.doc, answers: r.answers.map(([p, l]) => {
    const st = clients[r.doc].getStackContext(p, ["L" + l])["L" + l];
    return [p, l, st ? st.items.map((m) => [m.pos, m.refType]) : []];
}) }));
process.stdout.write(out.join("\n") + "\n");
