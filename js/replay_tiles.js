"use strict";
// findTile through the Node surface: the tiles_* logs replayed into BatchClients (tile labels on
// property key <tileKey> as "referenceTileLabels" arrays, js/mtlog.js), then every query of the
// reference's fixture asked with BatchClient.findTile; one JSON line per document {doc, answers}.
//   node replay_tiles.js <log.mtlog> <tiles.expected.jsonl> <logName> [tileKey]
const fs = require("fs");
const { BatchEngine } = require("./batchClient.js");
const { loadLog, messages } = require("./mtlog.js");

const log = loadLog(process.argv[2]);
const rows = fs.readFileSync(process.argv[3], "utf8").split("\n").filter((x) => x.trim()).map((x) => JSON.parse(x))
    .filter((r) => r.log === process.argv[4]);
const tileKey = parseInt(process.argv[5] || "0", 10);
const eng = new BatchEngine({ maxDocs: log.nDocs, opsPerLaunch: 32 });
const clients = [];
for (let d = 0; d < log.nDocs; d++) {
    const c = eng.createClient();
    c.startOrUpdateCollaboration("observer");
    for (const m of messages(log, d, { tileKey })) c.applyMsg(m);
    clients.push(c);
}
const out = rows.map((r) => JSON.stringify({ doc: r.doc, answers: r.answers.map(([p, l, prec]) => {
    const t = clients[r.doc].findTile(p, "L" + l, prec === 1);
    return [p, l, prec, t ? t.pos : null];
}) }));
process.stdout.write(out.join("\n") + "\n");
