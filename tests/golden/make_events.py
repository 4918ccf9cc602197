#!/usr/bin/env python3
"""Regenerate tests/golden/events.jsonl FROM THE REFERENCE ITSELF (build container only).

For each op log below, oracle/tsref/replay_ref.js replays every document through a reference
observer Client with `mergeTreeDeltaCallback` and `mergeTreeMaintenanceCallback` attached
(mergeTreeDeltaCallback.ts:15-73) and writes the callbacks in the canonical event form
(fluidframework_amd/events.py).  Small logs keep the callbacks themselves; the synthetic logs keep
the callback count and a SHA-256 of their canonical JSON per document.  A document on which the
reference throws keeps only the callbacks of the messages before the failing one (the engine
halts before it; the reference half-applies it).
One JSON line per (log, document): {log, doc, n, sha256, events?}.
"""
import hashlib
import json
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))

FULL = ['scenarios', 'markers', 'errors', 'empty_inserts', 'wide']
DIGEST = ['synth_tiny', 'synth_c3', 'synth_c4', 'synth_markers', 'wide_synth']


def canonical(events):
    return json.dumps(events, separators=(',', ':'))


def main():
    subprocess.check_call([sys.executable, os.path.join(REPO, 'oracle/tsref/build_ref.py')])
    replay = os.path.join(REPO, 'oracle/tsref/replay_ref.js')
    errs = {}
    for name in FULL + DIGEST:  # the failing message's seq, from the reference's errstate fixtures
        with open(os.path.join(HERE, name + '.expected.jsonl')) as f:
            for line in f:
                r = json.loads(line)
                if r.get('err') is not None:
                    errs[(name, r['doc'])] = r['err_seq']
    out = []
    for name in FULL + DIGEST:
        path = os.path.join(HERE, name + '.mtlog')
        res = subprocess.run(['node', replay, 'events', path], check=True, capture_output=True, text=True)
        for line in res.stdout.strip().split('\n'):
            r = json.loads(line)
            ev = r['events']
            if (name, r['doc']) in errs:
                ev = [e for e in ev if e[0] < errs[(name, r['doc'])]]
            rec = {'log': name, 'doc': r['doc'], 'n': len(ev), 'sha256': hashlib.sha256(canonical(ev).encode()).hexdigest()}
            if name in FULL:
                rec['events'] = ev
            out.append(json.dumps(rec, separators=(',', ':')))
        print(name, 'done')
    with open(os.path.join(HERE, 'events.jsonl'), 'w') as f:
        f.write('\n'.join(out) + '\n')


if __name__ == '__main__':
    main()
