#!/usr/bin/env python3
"""Regenerate local_huge and local_offline (build container only): editing-client farm logs FROM
THE REFERENCE ITSELF beyond the editing form's LDS limits, for its HBM-workspace forms.  Same farm
and replay as make_local.py (oracle/tsref/local_farm.js, replay_ref.js `local`), 4 clients, c1
lagging:
  * local_huge: 2 documents, 32000 edits over all clients: they grow past 1024 segments;
  * local_offline: 6 documents, 3000 edits; c1 goes offline for 12-24 rounds now and then (its
    messages held, nothing delivered) so that 110-170 of its edits are pending at once (the
    reference client throws "MergeTree insert failed" on some such runs: the farm drops those);
  * local_offline_long: 3 documents, 1500 edits; c1 stays offline for 90-120 rounds at 3-7 edits a
    round, so 400-484 of its edits are pending at once (the farm caps them at 480 while it is away;
    runs in which the reference's own clients diverge are dropped).
    python tests/golden/make_local_huge.py [--only=local_offline_long]
<name>.expected.jsonl holds the reference Client c1's canonical state at 6 checkpoints and at the
end (one JSON line per document, like local.expected.jsonl); local_offline.events.jsonl the count and
SHA-256 of c1's delta callbacks per document (like local_events.jsonl)."""
import json
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
sys.path.insert(0, HERE)

from make_golden import build_log  # noqa: E402

LOGS = (('local_huge', 2, 22, 32000, 0), ('local_offline', 6, 33, 3000, 1), ('local_offline_long', 3, 44, 1500, 2))
# (name, docs, seed, edits over all clients, offline: 1 = sessions of 12-24 rounds, 2 = of 90-120 rounds
# with up to 480 of c1's edits pending); 4 clients, c1 lagging, 6 checkpoints
N_CLIENTS, PARTIAL, N_CK = 4, 1, 6


def main():
    subprocess.check_call([sys.executable, os.path.join(REPO, 'oracle/tsref/build_ref.py')])
    only = [a.split('=', 1)[1] for a in sys.argv[1:] if a.startswith('--only=')]
    for name, n_docs, seed, n_ops, offline in LOGS:
        if not only or name in only[0].split(','):
            make(name, n_docs, seed, n_ops, offline)


def make(name, n_docs, seed, n_ops, offline):
    farm = os.path.join(REPO, 'oracle/tsref/local_farm.js')
    replay = os.path.join(REPO, 'oracle/tsref/replay_ref.js')
    res = subprocess.run(['node', farm, str(n_docs), str(seed), str(n_ops), str(N_CLIENTS), str(PARTIAL), '0', '0',
                          str(offline)], check=True, capture_output=True, text=True)
    docs = [[(s, r, m, c, t, p1, p2, text, None if props is None else {int(k): v for k, v in props.items()}, flags)
             for (s, r, m, c, t, p1, p2, text, props, flags) in recs] for recs in json.loads(res.stdout)['docs']]
    path = os.path.join(HERE, name + '.mtlog')
    build_log(docs).save(path)
    res = subprocess.run(['node', replay, 'local', path, str(N_CK)], check=True, capture_output=True, text=True)
    out = []
    for line in res.stdout.strip().split('\n'):
        r = json.loads(line)
        assert r['err'] is None, r['err']
        out.append(json.dumps(dict(log=name, **r), separators=(',', ':')))
        print(name, 'doc', r['doc'], 'segments at the checkpoints', [len(st['segs']) for _, st in r['states']])
    with open(os.path.join(HERE, name + '.expected.jsonl'), 'w') as f:
        f.write('\n'.join(out) + '\n')
    if offline:  # the reference client's callbacks (as make_local.py's local_events.jsonl): count + SHA-256
        import hashlib
        res = subprocess.run(['node', replay, 'localevents', path], check=True, capture_output=True, text=True)
        ev_out = []
        for line in res.stdout.strip().split('\n'):
            r = json.loads(line)
            assert r['err'] is None, r['err']
            ev = r['events']
            ev_out.append(json.dumps(dict(log=name, doc=r['doc'], n=len(ev), sha256=hashlib.sha256(
                json.dumps(ev, separators=(',', ':')).encode()).hexdigest()), separators=(',', ':')))
        with open(os.path.join(HERE, name + '.events.jsonl'), 'w') as f:
            f.write('\n'.join(ev_out) + '\n')


if __name__ == '__main__':
    main()
