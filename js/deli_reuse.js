"use strict";
// 200 sessions of one document, each a join, two ops and a leave (Fluid gives every connection
// a new client id): short ids are given back by the leaves and reused (deliSequencer.js), so no
// 64-client limit is hit; every op is sent.  Also a leave of a never-seen client (dropped, no
// id interned).  Prints {statuses, seq, interned}.
const { DeliSequencer } = require("./deliSequencer.js");

function factory(clientId) {
    let csn = 0;
    return {
        create: (ref) => ({ clientId, type: "RawOperation",
            operation: { clientSequenceNumber: ++csn, contents: null, referenceSequenceNumber: ref, type: "op" } }),
        join: () => ({ clientId: null, type: "RawOperation",
            operation: { clientSequenceNumber: -1, contents: null, referenceSequenceNumber: -1, type: "join",
                data: JSON.stringify({ clientId, detail: { mode: "write", scopes: [] } }) } }),
        leave: () => ({ clientId: null, type: "RawOperation",
            operation: { clientSequenceNumber: -1, contents: null, referenceSequenceNumber: -1, type: "leave",
                data: JSON.stringify(clientId) } }),
    };
}
const dl = new DeliSequencer({ maxDocs: 1 });
const statuses = {};
let seq = 0;
const count = (res) => res[0].forEach((r) => {
    statuses[r.status] = (statuses[r.status] || 0) + 1;
    if (r.sequenceNumber !== undefined) seq = Math.max(seq, r.sequenceNumber);
});
dl.queue(0, factory("ghost").leave());
for (let s = 0; s < 200; s++) {
    const f = factory("session-" + s);
    dl.queue(0, f.join());               // sequenced 4s + 1: each session revs 4 times
    dl.queue(0, f.create(4 * s + 1));    // refSeq = the join's seq, >= the msn the joiner entered at
    dl.queue(0, f.create(4 * s + 1));
    dl.queue(0, f.leave());
    if (s % 10 === 9) count(dl.flush());
}
console.log(JSON.stringify({ statuses, seq, interned: dl.ids[0].size }));
