#!/usr/bin/env python3
"""In-callback read fixtures FROM THE REFERENCE ITSELF (build container only; needs /root/reference and node).

What a SharedString user's delta listener reads INSIDE the callback (mergeTree.ts:1981-1988 fires it in
the middle of the apply): SharedString.getText() (textHelper.getText at the client's collab window,
sequence.ts), getLength() and getPosition(segment) of every delta segment.  oracle/tsref/replay_ref.js
`seqreads` replays each log on a reference Client (the editing client "c1" of a local_* / seqdelta log,
else the observer) and records [seq (-1: local edit), text, length, [position, ...]] per callback.
The engine side (js/replay_local.js `seqreads`, BatchEngine syncCallbacks) must read the same.

seqreads.expected.jsonl: {log, doc, err, n, reads} in full for seqdelta.mtlog (sequenceDeltaEvent.spec.ts
re-expressed, make_seqdelta.py) and {log, doc, err, n, sha256} (of the canonical read list) for the
first documents of a few editing / observer logs.  Fixtures are data only (inputs and reference outputs).
"""
import hashlib
import json
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))

# (log, first documents)
LOGS = (('seqdelta', None), ('local_lag', 6), ('local_rounds', 6), ('local_markers', 4), ('scenarios', 12))


def main():
    subprocess.check_call([sys.executable, os.path.join(REPO, 'oracle/tsref/build_ref.py')])
    replay = os.path.join(REPO, 'oracle/tsref/replay_ref.js')
    out = []
    for name, n in LOGS:
        cmd = ['node', replay, 'seqreads', os.path.join(HERE, name + '.mtlog')] + ([str(n)] if n else [])
        res = subprocess.run(cmd, check=True, capture_output=True, text=True)
        for line in res.stdout.strip().split('\n'):
            r = json.loads(line)
            row = {'log': name, 'doc': r['doc'], 'err': r['err'], 'n': len(r['reads'])}
            if name == 'seqdelta':
                row['reads'] = r['reads']
            else:
                row['sha256'] = hashlib.sha256(json.dumps(r['reads'], separators=(',', ':')).encode()).hexdigest()
            out.append(row)
    with open(os.path.join(HERE, 'seqreads.expected.jsonl'), 'w') as f:
        f.write('\n'.join(json.dumps(r, separators=(',', ':')) for r in out) + '\n')
    print(len(out), 'rows', os.path.getsize(os.path.join(HERE, 'seqreads.expected.jsonl')), 'B')


if __name__ == '__main__':
    main()
