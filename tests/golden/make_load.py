#!/usr/bin/env python3
"""Snapshot-load fixtures (load half) FROM THE REFERENCE ITSELF.

Runs in the build container only (needs /root/reference and node):
  1. load_<set>.jsonl -- for every document of a committed op log: messages [0, k) replayed on a
     reference observer, its SnapshotV1 tree emitted, that tree loaded into a fresh reference
     Client through SnapshotLoader (snapshotLoader.ts:35-225), messages [k, n) applied to it
     (oracle/tsref/replay_ref.js `load`).  Stored: the emitted snapshot (input) and the loaded
     client's final canonical state and error (expected output).
  2. ref_snapshots/ -- the reference's own snapshot test data (packages/dds/sequence/src/test/
     snapshots/{v1,legacy,legacyWithCatchUp}/*.json, all 15 data files the reference's snapshotVersion
     spec loads; text, a large body, annotated text and markers), and expected.jsonl: the
     reference loader's state after loading each and applying ref_followup.mtlog (the spec's
     edits -- NEWTEXT every 50 characters, a replace of everything, a remove of everything --
     as sequenced remote ops).
Fixtures are data only (inputs and reference outputs).
"""
import json
import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
sys.path.insert(0, HERE)

from make_golden import I, R, build_log  # noqa: E402

REF_SNAP = '/root/reference/packages/dds/sequence/src/test/snapshots'
# (set, message index k, mergeTreeSnapshotChunkSize (0 = default))
LOG_SETS = [('synth_tiny', 384, 0), ('synth_c3', 256, 300), ('synth_c4', 512, 0), ('scenarios', 3, 0),
            ('synth_c1', 1024, 400), ('markers', 4, 0), ('synth_markers', 320, 250),
            ('wide_many', 330, 200), ('wide_xl', 130, 200)]
# every data file snapshotVersion.spec.ts loads (sequence/src/test/snapshots/{v1,legacy,legacyWithCatchUp}/*)
REF_FILES = [f'{v}/{k}' for v in ('v1', 'legacy', 'legacyWithCatchUp')
             for k in ('headerOnly', 'headerAndBody', 'largeBody', 'withAnnotations', 'withMarkers')]


def followup(length, seq0=0):
    """snapshotVersion.spec.ts:53-73 as remote ops of client c1 (each sees everything before it)."""
    ops, s, n = [], seq0, length
    for j in range(0, 1 << 30, 50):
        if j >= n:
            break
        s += 1
        ops.append(I(s, s - 1, max(seq0, s - 8), 1, j, 'NEWTEXT'))
        n += 7
    s += 1
    ops.append(R(s, s - 1, s - 2, 2, 0, n))          # replaceText(0, len, "hello world"): remove ...
    s += 1
    ops.append(I(s, s - 1, s - 2, 2, 0, 'hello world'))  # ... then insert
    s += 1
    ops.append(R(s, s - 1, s - 1, 1, 0, 11))         # removeText(0, len)
    return ops


def main():
    subprocess.check_call([sys.executable, os.path.join(REPO, 'oracle/tsref/build_ref.py')])
    replay = os.path.join(REPO, 'oracle/tsref/replay_ref.js')
    only = sys.argv[1:]  # (regenerate just these sets)
    for name, k, chunk in LOG_SETS:
        if only and name not in only:
            continue
        args = ['node', replay, 'load', os.path.join(HERE, name + '.mtlog'), str(k)] + ([str(chunk)] if chunk else [])
        res = subprocess.run(args, check=True, capture_output=True, text=True)
        out = os.path.join(HERE, f'load_{name}.jsonl')
        with open(out, 'w') as f:
            for line in res.stdout.strip().split('\n'):
                r = json.loads(line)
                r['k'] = k
                f.write(json.dumps(r, separators=(',', ':')) + '\n')
        print(os.path.basename(out), os.path.getsize(out), 'B')
    if only:
        return
    dst = os.path.join(HERE, 'ref_snapshots')
    os.makedirs(dst, exist_ok=True)
    lines = []
    for rel in REF_FILES:
        src = os.path.join(REF_SNAP, rel + '.json')
        fn = rel.replace('/', '_') + '.json'
        shutil.copyfile(src, os.path.join(dst, fn))
        # the loaded length decides the follow-up edits
        res = subprocess.run(['node', replay, 'loadtree', src], check=True, capture_output=True, text=True)
        st = json.loads(res.stdout)['state']
        length = sum(1 if isinstance(s[0], dict) else len(s[0]) for s in st['segs'] if s[3] == -1)
        log = build_log([followup(length, st['seq'])])
        logf = os.path.join(dst, fn.replace('.json', '.mtlog'))
        log.save(logf)
        res = subprocess.run(['node', replay, 'loadtree', src, logf], check=True, capture_output=True, text=True)
        r = json.loads(res.stdout)
        r['file'] = fn
        r['loaded'] = st
        lines.append(json.dumps(r, separators=(',', ':')))
        print(fn, 'length', length, 'ops', log.n_ops, 'err', r['err'])
    with open(os.path.join(dst, 'expected.jsonl'), 'w') as f:
        f.write('\n'.join(lines) + '\n')


if __name__ == '__main__':
    main()
