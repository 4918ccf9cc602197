"use strict";
// Replays the scenarios of the reference's deli tests (lambda.spec.ts:101-248) as
// IRawOperationMessages (built the way test-utils/src/messageFactory.ts:90-131 builds them)
// through DeliSequencer, one document per scenario; prints one JSON line per document.
const { DeliSequencer } = require("./deliSequencer.js");

function factory(clientId) {
    let csn = 0;
    return {
        create: (ref = 0) => ({ clientId, type: "RawOperation",
            operation: { clientSequenceNumber: ++csn, contents: null, referenceSequenceNumber: ref, type: "op" } }),
        createJoin: () => ({ clientId: null, type: "RawOperation",
            operation: { clientSequenceNumber: -1, contents: null, referenceSequenceNumber: -1, type: "join",
                data: JSON.stringify({ clientId, detail: { mode: "write", scopes: [] } }) } }),
        createLeave: () => ({ clientId: null, type: "RawOperation",
            operation: { clientSequenceNumber: -1, contents: null, referenceSequenceNumber: -1, type: "leave",
                data: JSON.stringify(clientId) } }),
    };
}

const scenarios = [];
{   // "Should remove clients after a disconnect" (:193-247)
    const a = factory("quiet-rat"), b = factory("test2"), c = factory("test3");
    scenarios.push([a.createJoin(), b.createJoin(), a.create(1), b.create(2), a.createLeave(), b.create(4),
        b.createLeave(), c.createJoin(), c.create(7)]);
}
{   // "Should ticket new clients connecting above msn" (:149-167)
    const a = factory("quiet-rat"), b = factory("test2");
    scenarios.push([a.createJoin(), a.create(10), a.create(20), b.createJoin(), b.create(25), a.create(22)]);
}
{   // forceNack + "Should nack all future messages from a nacked client" (:57-69, 117-128)
    const a = factory("quiet-rat"), b = factory("test2");
    scenarios.push([a.createJoin(), a.create(10), b.createJoin(), b.create(5), b.create(15)]);
}
const dl = new DeliSequencer({ maxDocs: scenarios.length });
scenarios.forEach((s, d) => s.forEach((m) => dl.queue(d, m)));
const out = dl.flush();
out.forEach((res, d) => console.log(JSON.stringify(res.map((r) => [r.status, r.sequenceNumber === undefined ? null :
    r.sequenceNumber, r.minimumSequenceNumber === undefined ? null : r.minimumSequenceNumber,
    r.nack ? r.nack.reason : null]))));
