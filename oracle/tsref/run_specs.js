"use strict";
// Runs the reference's own merge-tree unit specs against the transpiled reference in
// oracle/_tsref (test infrastructure: validates the type-strip before the oracle is trusted).
const path = require("path");
const root = path.join(__dirname, "..", "_tsref");
const shim = require(path.join(root, "mocha_shim.js"));
const names = process.argv.slice(2);
// (a name with a "/" is relative to oracle/_tsref, e.g. sequence/src/test/sequenceDeltaEvent.spec)
const files = names.map((n) => path.join(root, n.includes("/") ? "" : "merge-tree/src/test", n.endsWith(".js") ? n : n + ".js"));
shim.run(files).then((res) => {
  let pass = 0, fail = 0, skip = 0;
  for (const r of res) {
    if (r.status === "pass") pass++; else if (r.status === "skip") skip++;
    else { fail++; console.log("FAIL", r.name, "\n   ", r.error.split("\n").slice(0, 4).join("\n    ")); }
  }
  console.log(JSON.stringify({ pass, fail, skip }));
  process.exit(fail ? 1 : 0);
});
