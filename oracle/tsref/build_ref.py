#!/usr/bin/env python3
"""Build the runnable reference oracle `oracle/_tsref/` from /root/reference (this container only).

TEST INFRASTRUCTURE ONLY (see oracle/README.md).  Type-strips (tsstrip.py) exactly the
reference files the observer apply path needs -- packages/dds/merge-tree/src/*.ts and its
test harness (TestClient, farm runner, the unit-test specs), and the sequence package's
SequenceDeltaEvent (sequenceDeltaEvent.ts, the delta-event wrapper) -- plus the two helpers it uses
from @fluidframework/common-utils (assert.ts:12-16, trace.ts:12-31), the protocol enums
(protocol-definitions/src/protocol.ts) and test-runtime-utils' MockStorage.  Everything else
the imports name (loggers, container enums, base64, random-js for the farm specs) gets a small
stub written here; the stubs carry no merge-tree logic.

Output goes to oracle/_tsref/ which is git-ignored and gpurun-ignored: the reference never
enters the repository history and never travels to the GPU box.
"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from tsstrip import strip_file  # noqa: E402

REF = os.environ.get('FLUID_REFERENCE', '/root/reference')
OUT = os.path.join(os.path.dirname(HERE), '_tsref')
MT = os.path.join(REF, 'packages/dds/merge-tree/src')

STUBS = {
    'node_modules/@fluidframework/common-utils/index.js': r'''
"use strict";
const { performance } = require("perf_hooks");
exports.performance = performance;
Object.assign(exports, require("./assert"));
Object.assign(exports, require("./trace"));
exports.fromBase64ToUtf8 = (s) => Buffer.from(s, "base64").toString("utf8");
exports.fromUtf8ToBase64 = (s) => Buffer.from(s, "utf8").toString("base64");
exports.IsoBuffer = Buffer;
exports.unreachableCase = (x) => { throw new Error(`unreachable ${x}`); };
''',
    'node_modules/@fluidframework/common-utils/indexNode.js': r'''
"use strict";
exports.performance = require("perf_hooks").performance;
''',
    'node_modules/@fluidframework/protocol-definitions/index.js': r'''
"use strict";
Object.assign(exports, require("./protocol"));
exports.TreeEntry = { Blob: "Blob", Commit: "Commit", Tree: "Tree", Attachment: "Attachment" };
exports.FileMode = { File: "100644", Executable: "100755", Directory: "040000", Symlink: "120000" };
''',
    'node_modules/@fluidframework/telemetry-utils/index.js': r'''
"use strict";
class NullLogger {
  send() {} sendTelemetryEvent() {} sendErrorEvent() {} sendPerformanceEvent() {}
  logGenericError() {} logException() {} debugAssert() {} shipAssert() {}
}
exports.DebugLogger = { create: () => new NullLogger(), mixinDebugLogger: (l) => l || new NullLogger() };
exports.ChildLogger = { create: (l) => l || new NullLogger() };
''',
    'node_modules/@fluidframework/container-definitions/index.js': r'''
"use strict";
exports.AttachState = { Detached: "Detached", Attaching: "Attaching", Attached: "Attached" };
''',
    'node_modules/@fluidframework/runtime-utils/index.js': r'''
"use strict";
exports.listBlobsAtTreePath = async function (tree, path) {
  const parts = path.split("/").filter((p) => p.length > 0);
  let t = tree;
  for (const p of parts) {
    const e = t && t.entries.find((x) => x.path === p && x.type === "Tree");
    if (!e) { return []; }
    t = e.value;
  }
  return t.entries.filter((e) => e.type === "Blob").map((e) => e.path);
};
''',
    # the sequence package's SequenceDeltaEvent (sequenceDeltaEvent.ts) imports the merge-tree by name
    'node_modules/@fluidframework/merge-tree/index.js': r'''
"use strict";
module.exports = require("../../../merge-tree/src/index.js");
''',
    'node_modules/@fluidframework/merge-tree/dist/test/index.js': r'''
"use strict";
module.exports = require("../../../../../merge-tree/src/test/index.js");
''',
    'node_modules/@fluidframework/test-runtime-utils/index.js': r'''
"use strict";
Object.assign(exports, require("./mockStorage"));
''',
    # random-js 1.0.8 API subset used by the farm specs (engines.mt19937, integer).  The farms
    # pin convergence only, so only the API shape matters, not the exact stream.
    'node_modules/random-js/index.js': r'''
"use strict";
function mt19937() {
  const mt = new Uint32Array(624); let idx = 625;
  function init(s) { mt[0] = s >>> 0; for (let i = 1; i < 624; i++) { const p = mt[i - 1] ^ (mt[i - 1] >>> 30);
    mt[i] = ((((p & 0xffff0000) >>> 16) * 1812433253) << 16) + (p & 0x0000ffff) * 1812433253 + i; } idx = 624; }
  function gen() { if (idx >= 624) { if (idx === 625) init(5489); for (let k = 0; k < 624; k++) {
      const y = (mt[k] & 0x80000000) | (mt[(k + 1) % 624] & 0x7fffffff);
      mt[k] = mt[(k + 397) % 624] ^ (y >>> 1) ^ ((y & 1) ? 0x9908b0df : 0); } idx = 0; }
    let y = mt[idx++]; y ^= y >>> 11; y ^= (y << 7) & 0x9d2c5680; y ^= (y << 15) & 0xefc60000; return (y ^ (y >>> 18)) >>> 0; }
  const eng = () => gen() | 0;
  eng.seed = (s) => { init(s); return eng; };
  eng.seedWithArray = (key) => { init(19650218); let i = 1, j = 0; const n = key.length;
    for (let k = Math.max(624, n); k > 0; k--) { const p = mt[i - 1] ^ (mt[i - 1] >>> 30);
      mt[i] = ((mt[i] ^ (((((p & 0xffff0000) >>> 16) * 1664525) << 16) + ((p & 0x0000ffff) * 1664525))) + (key[j] >>> 0) + j) >>> 0;
      i++; j++; if (i >= 624) { mt[0] = mt[623]; i = 1; } if (j >= n) j = 0; }
    for (let k = 623; k > 0; k--) { const p = mt[i - 1] ^ (mt[i - 1] >>> 30);
      mt[i] = ((mt[i] ^ (((((p & 0xffff0000) >>> 16) * 1566083941) << 16) + (p & 0x0000ffff) * 1566083941)) - i) >>> 0;
      i++; if (i >= 624) { mt[0] = mt[623]; i = 1; } }
    mt[0] = 0x80000000; idx = 624; return eng; };
  return eng;
}
function integer(min, max) { const range = max - min + 1;
  return (engine) => min + Math.floor(((engine() >>> 0) / 4294967296) * range); }
function real(min, max) { return (engine) => min + ((engine() >>> 0) / 4294967296) * (max - min); }
function bool() { return (engine) => ((engine() >>> 0) & 1) === 1; }
function pick(engine, arr) { return arr[integer(0, arr.length - 1)(engine)]; }
function string(pool) { pool = pool || "abcdefghijklmnopqrstuvwxyzABCDEFGHIJKLMNOPQRSTUVWXYZ0123456789_-";
  return (engine, len) => { let s = ""; for (let i = 0; i < len; i++) s += pool[integer(0, pool.length - 1)(engine)]; return s; }; }
const random = { engines: { mt19937, nativeMath: () => (Math.random() * 4294967296) | 0 }, integer, real, bool, pick, string };
module.exports = random; module.exports.default = random;
''',
}

MOCHA_SHIM = r'''
"use strict";
// Minimal mocha-compatible runner for the transpiled reference specs (test infrastructure).
const suites = [];
let cur = { name: "", tests: [], before: [], beforeEach: [], after: [], afterEach: [], children: [], parent: null };
const root = cur;
global.describe = (name, fn) => { const s = { name, tests: [], before: [], beforeEach: [], after: [], afterEach: [], children: [], parent: cur };
  cur.children.push(s); const p = cur; cur = s; fn(); cur = p; return { timeout() { return this; } }; };
global.describe.skip = () => {};
global.it = (name, fn) => { const t = { name, fn, skip: false }; cur.tests.push(t); return { timeout() { return this; } }; };
global.it.skip = (name) => { cur.tests.push({ name, fn: null, skip: true }); return { timeout() { return this; } }; };
global.before = (fn) => cur.before.push(fn); global.beforeEach = (fn) => cur.beforeEach.push(fn);
global.after = (fn) => cur.after.push(fn); global.afterEach = (fn) => cur.afterEach.push(fn);
function chain(s, key) { const out = []; for (let x = s; x; x = x.parent) out.unshift(...x[key]); return out; }
async function runSuite(s, path, res) {
  for (const f of s.before) await f.call({ timeout() {} });
  for (const t of s.tests) {
    const full = path.concat([t.name]).join(" / ");
    if (t.skip) { res.push({ name: full, status: "skip" }); continue; }
    try { for (const f of chain(s, "beforeEach")) await f.call({ timeout() {} });
      await t.fn.call({ timeout() {} }); for (const f of chain(s, "afterEach")) await f.call({});
      res.push({ name: full, status: "pass" }); }
    catch (e) { res.push({ name: full, status: "fail", error: String(e && e.stack || e) }); }
  }
  for (const c of s.children) await runSuite(c, path.concat([c.name]), res);
  for (const f of s.after) await f.call({});
}
exports.run = async function (files) { for (const f of files) require(f); const res = []; await runSuite(root, [], res); return res; };
'''


def strip_to(src_path, dst_path):
    with open(src_path) as f:
        src = f.read()
    js = strip_file(src, src_path)
    os.makedirs(os.path.dirname(dst_path), exist_ok=True)
    with open(dst_path, 'w') as f:
        f.write(js)


def main():
    if not os.path.isdir(MT):
        print(f'reference not found at {REF}; skipping oracle/_tsref build')
        return 1
    for name in sorted(os.listdir(MT)):
        if name.endswith('.ts'):
            strip_to(os.path.join(MT, name), os.path.join(OUT, 'merge-tree/src', name[:-3] + '.js'))
    for name in sorted(os.listdir(os.path.join(MT, 'test'))):
        if name.endswith('.ts'):
            strip_to(os.path.join(MT, 'test', name), os.path.join(OUT, 'merge-tree/src/test', name[:-3] + '.js'))
    strip_to(os.path.join(REF, 'packages/dds/sequence/src/sequenceDeltaEvent.ts'),
             os.path.join(OUT, 'sequence/src/sequenceDeltaEvent.js'))
    strip_to(os.path.join(REF, 'packages/dds/sequence/src/test/sequenceDeltaEvent.spec.ts'),
             os.path.join(OUT, 'sequence/src/test/sequenceDeltaEvent.spec.js'))
    cu = os.path.join(REF, 'common/lib/common-utils/src')
    strip_to(os.path.join(cu, 'assert.ts'), os.path.join(OUT, 'node_modules/@fluidframework/common-utils/assert.js'))
    strip_to(os.path.join(cu, 'trace.ts'), os.path.join(OUT, 'node_modules/@fluidframework/common-utils/trace.js'))
    strip_to(os.path.join(REF, 'server/routerlicious/packages/protocol-definitions/src/protocol.ts'),
             os.path.join(OUT, 'node_modules/@fluidframework/protocol-definitions/protocol.js'))
    strip_to(os.path.join(REF, 'packages/runtime/test-runtime-utils/src/mockStorage.ts'),
             os.path.join(OUT, 'node_modules/@fluidframework/test-runtime-utils/mockStorage.js'))
    for rel, text in STUBS.items():
        p = os.path.join(OUT, rel)
        os.makedirs(os.path.dirname(p), exist_ok=True)
        with open(p, 'w') as f:
            f.write(text.lstrip())
    with open(os.path.join(OUT, 'mocha_shim.js'), 'w') as f:
        f.write(MOCHA_SHIM.lstrip())
    print(f'built {OUT}')
    return 0


if __name__ == '__main__':
    sys.exit(main())
