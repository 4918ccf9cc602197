"use strict";
// An editing client through the Node surface: each document of a local_* log (tests/golden/
// make_local.py) replayed into a BatchClient "c<own>" -- its local edits through insertTextLocal /
// removeRangeLocal / annotateRangeLocal, the sequenced stream (its own messages = acks) through
// applyMsg -- one JSON line per document {doc, err, state}.
//   node replay_local.js <log.mtlog>
const { BatchEngine } = require("./batchClient.js");
const { loadLog, messages } = require("./mtlog.js");

const log = loadLog(process.argv[2]);
const eng = new BatchEngine({ maxDocs: log.nDocs, opsPerLaunch: 16 });
const clients = [];
for (let d = 0; d < log.nDocs; d++) {
    const items = [...messages(log, d)];
    const own = items.find((x) => x.local);
    const c = eng.createClient();
    c.startOrUpdateCollaboration(own ? "c" + own.client : "observer");
    for (const it of items) {
        if (!it.local) {
            c.applyMsg(it);
            continue;
        }
        const op = it.op;
        let r;
        if (op.type === 0) {
            r = typeof op.seg === "string" ? c.insertTextLocal(op.pos1, op.seg)
                : op.seg.marker ? c.insertMarkerLocal(op.pos1, op.seg.marker.refType, op.seg.props)
                    : c.insertTextLocal(op.pos1, op.seg.text, op.seg.props);
        } else if (op.type === 1) {
            r = c.removeRangeLocal(op.pos1, op.pos2);
        } else {
            r = c.annotateRangeLocal(op.pos1, op.pos2, op.props, op.combiningOp);
        }
        if (!r) throw new Error("local edit rejected");
    }
    clients.push(c);
}
const out = clients.map((c, d) => {
    let err = null, state = null;
    try { state = c.getState(); } catch (e) { err = String(e.message || e); }
    return JSON.stringify({ doc: d, err, state });
});
process.stdout.write(out.join("\n") + "\n");
