#!/usr/bin/env python3
"""Regenerate local_huge (build container only): an editing-client farm log FROM THE REFERENCE
ITSELF whose documents grow past 1024 segments (the editing form's LDS capacity), for the
editing form's HBM-workspace classes.  Same farm and replay as make_local.py (oracle/tsref/
local_farm.js, replay_ref.js `local`): 2 documents, 4 clients, c1 lagging, 32000 edits over all
clients; local_huge.expected.jsonl holds the reference Client c1's canonical state at 6 checkpoints
and at the end (one JSON line per document, like local.expected.jsonl)."""
import json
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
sys.path.insert(0, HERE)

from make_golden import build_log  # noqa: E402

N_DOCS, SEED, N_OPS, N_CLIENTS, PARTIAL, N_CK = 2, 22, 32000, 4, 1, 6


def main():
    subprocess.check_call([sys.executable, os.path.join(REPO, 'oracle/tsref/build_ref.py')])
    farm = os.path.join(REPO, 'oracle/tsref/local_farm.js')
    replay = os.path.join(REPO, 'oracle/tsref/replay_ref.js')
    res = subprocess.run(['node', farm, str(N_DOCS), str(SEED), str(N_OPS), str(N_CLIENTS), str(PARTIAL), '0', '0'],
                         check=True, capture_output=True, text=True)
    docs = [[(s, r, m, c, t, p1, p2, text, None if props is None else {int(k): v for k, v in props.items()}, flags)
             for (s, r, m, c, t, p1, p2, text, props, flags) in recs] for recs in json.loads(res.stdout)['docs']]
    path = os.path.join(HERE, 'local_huge.mtlog')
    build_log(docs).save(path)
    res = subprocess.run(['node', replay, 'local', path, str(N_CK)], check=True, capture_output=True, text=True)
    out = []
    for line in res.stdout.strip().split('\n'):
        r = json.loads(line)
        assert r['err'] is None, r['err']
        out.append(json.dumps(dict(log='local_huge', **r), separators=(',', ':')))
        print('doc', r['doc'], 'segments at the checkpoints', [len(st['segs']) for _, st in r['states']])
    with open(os.path.join(HERE, 'local_huge.expected.jsonl'), 'w') as f:
        f.write('\n'.join(out) + '\n')


if __name__ == '__main__':
    main()
