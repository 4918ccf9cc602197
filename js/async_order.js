"use strict";
// Two flushAsync() calls issued back to back without awaiting, then a synchronous getText():
// the addon's turnstile must apply the batches in flush order, each exactly once, and the
// readout must see both (mtgpu_napi.c engine_box).  Prints {text, length, seq}.
const { BatchEngine } = require("./batchClient.js");

const eng = new BatchEngine({ maxDocs: 4, opsPerLaunch: 8 });
const cs = [0, 1, 2, 3].map(() => { const c = eng.createClient(); c.startOrUpdateCollaboration("observer"); return c; });
let seq = 0;
const promises = [];
for (let round = 0; round < 6; round++) {
    for (const c of cs) {
        for (let k = 0; k < 5; k++) {
            seq++;
            c.insertTextRemote(0, String.fromCharCode(97 + (seq % 26)), undefined, seq, seq - 1, "w" + (k % 3));
        }
    }
    promises.push(eng.flushAsync());   // not awaited
}
const text = cs.map((c) => c.getText());
Promise.all(promises).then(() => {
    console.log(JSON.stringify({ text, length: cs.map((c) => c.getLength()), seq }));
});
