"use strict";
// Snapshot load through the Node surface (js/snapshotLoader.js over mt_docs_load), for the tests:
//   node replay_load.js sets <load_X.jsonl> <X.mtlog> [opsPerLaunch]
//       every row's snapshot loaded into its document's BatchClient, then the log's messages from
//       the row's k-th on; one JSON line per document {doc, err, state (long ids, real prop names)}
//   node replay_load.js files <expected.jsonl> <dir>
//       the reference's own snapshot files (sequence/src/test/snapshots) loaded one per client, then
//       the edits of <file>.mtlog; lines {file, loaded, err, state}
const fs = require("fs");
const path = require("path");
const { BatchEngine } = require("./batchClient.js");
const { loadSnapshots } = require("./snapshotLoader.js");
const { loadLog, messages } = require("./mtlog.js");

function readJsonl(f) {
    return fs.readFileSync(f, "utf8").split("\n").filter((x) => x.trim()).map((x) => JSON.parse(x));
}

function applyAll(client, msgs) {
    try {
        for (const m of msgs) client.applyMsg(m);
        client.getLength();  // flush + the document's error, if any
    } catch (e) {
        return String(e.message || e);
    }
    return null;
}

const mode = process.argv[2];
if (mode === "sets") {
    const rows = readJsonl(process.argv[3]);
    const log = loadLog(process.argv[4]);
    const eng = new BatchEngine({ maxDocs: log.nDocs, opsPerLaunch: parseInt(process.argv[5] || "0", 10) });
    const clients = [];
    for (let d = 0; d < log.nDocs; d++) {
        const c = eng.createClient();
        c.startOrUpdateCollaboration("observer");
        clients.push(c);
    }
    loadSnapshots(eng, rows.map((r) => ({ client: clients[r.doc], snapshot: r.snapshot })));
    const out = [];
    for (const r of rows) {
        const c = clients[r.doc];
        const err = applyAll(c, Array.from(messages(log, r.doc)).slice(r.k));
        out.push(JSON.stringify({ doc: r.doc, err, state: c.getState() }));
    }
    process.stdout.write(out.join("\n") + "\n");
} else if (mode === "files") {
    const cases = readJsonl(process.argv[3]);
    const dir = process.argv[4];
    // (an 88,890-character segment; the follow-up edits split the large bodies into thousands of segments)
    const eng = new BatchEngine({ maxDocs: cases.length, opsPerLaunch: 32, textCapacity: 512 * 1024, segCapacity: 8192 });
    const clients = cases.map(() => {
        const c = eng.createClient();
        c.startOrUpdateCollaboration("observer");
        return c;
    });
    const catchup = loadSnapshots(eng, cases.map((c, i) => ({ client: clients[i],
        snapshot: JSON.parse(fs.readFileSync(path.join(dir, c.file), "utf8")) })));
    const loaded = clients.map((c) => c.getState());
    const out = cases.map((c, i) => {
        const log = loadLog(path.join(dir, c.file.replace(".json", ".mtlog")));
        const err = applyAll(clients[i], catchup[i].concat(Array.from(messages(log, 0))));
        return JSON.stringify({ file: c.file, loaded: loaded[i], err, state: clients[i].getState() });
    });
    process.stdout.write(out.join("\n") + "\n");
} else if (mode === "markers") {
    // getMarkerFromId (client.ts:311-313) after loading the reference's snapshot files: every markerId
    // of the loaded state, then an id that is not there; lines {file, found: [[id, ordinal, position,
    // refType] | [id, null], ...]}
    const cases = readJsonl(process.argv[3]);
    const dir = process.argv[4];
    const eng = new BatchEngine({ maxDocs: cases.length, opsPerLaunch: 32, textCapacity: 512 * 1024, segCapacity: 8192 });
    const clients = cases.map(() => {
        const c = eng.createClient();
        c.startOrUpdateCollaboration("observer");
        return c;
    });
    loadSnapshots(eng, cases.map((c, i) => ({ client: clients[i],
        snapshot: JSON.parse(fs.readFileSync(path.join(dir, c.file), "utf8")) })));
    const out = cases.map((c, i) => {
        const ids = [];
        for (const s of clients[i].getState().segs) {
            if (s[0] !== null && typeof s[0] === "object" && s[6] && s[6].markerId !== undefined) ids.push(s[6].markerId);
        }
        ids.push("no such marker");
        const found = ids.map((id) => {
            const m = clients[i].getMarkerFromId(id);
            return m ? [id, m.ordinal, clients[i].getPosition(m), m.refType] : [id, null];
        });
        return JSON.stringify({ file: c.file, found });
    });
    process.stdout.write(out.join("\n") + "\n");
} else {
    throw new Error("mode: sets | files | markers");
}
