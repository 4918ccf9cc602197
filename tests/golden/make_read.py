#!/usr/bin/env python3
"""Read-surface fixtures FROM THE REFERENCE ITSELF (build container only; needs /root/reference and node).

VERDICT r02 "missing" #5: the Client read surface SharedString uses on applied state --
getContainingSegment / getPropertiesAtPosition / getRangeExtentsOfPosition (client.ts:1004-1040),
getPosition (:290), walkSegments (:275), resolveRemoteClientPosition (:838-847).
oracle/tsref/replay_ref.js `read` replays each document of a committed log on a reference Client (the
editing client "c<own>" of a local_* log, else the observer) and queries its final state: the three
position queries at up to ~50 positions (0 .. length + 1), four walkSegments ranges (one stopped by the
handler), getPosition of every leaf, and resolveRemoteClientPosition for up to four remote clients at
two refSeqs inside the collab window.  read.expected.jsonl: {log, ...the replay's line} in full for
the first documents of each log, {log, doc, sha256} of the canonical line for the others.
Fixtures are data only (inputs and reference outputs).
"""
import hashlib
import json
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
LOGS = ('scenarios', 'markers', 'synth_markers', 'wide', 'synth_c1', 'local_lag', 'local_markers', 'local_reconnect')
FULL_DOCS = 4


def main():
    subprocess.check_call([sys.executable, os.path.join(REPO, 'oracle/tsref/build_ref.py')])
    replay = os.path.join(REPO, 'oracle/tsref/replay_ref.js')
    out = []
    for name in LOGS:
        res = subprocess.run(['node', replay, 'read', os.path.join(HERE, name + '.mtlog')], check=True,
                             capture_output=True, text=True)
        for line in res.stdout.strip().split('\n'):
            r = json.loads(line)
            assert r['err'] is None, (name, r['doc'], r['err'])
            if r['doc'] < FULL_DOCS:
                out.append(json.dumps(dict(log=name, **r), separators=(',', ':')))
            else:
                h = hashlib.sha256(json.dumps(r, separators=(',', ':')).encode()).hexdigest()
                out.append(json.dumps(dict(log=name, doc=r['doc'], sha256=h), separators=(',', ':')))
    with open(os.path.join(HERE, 'read.expected.jsonl'), 'w') as f:
        f.write('\n'.join(out) + '\n')
    print(len(out), 'rows', os.path.getsize(os.path.join(HERE, 'read.expected.jsonl')), 'B')


if __name__ == '__main__':
    main()
