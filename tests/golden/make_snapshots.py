#!/usr/bin/env python3
"""Snapshot fixtures: every committed *.mtlog replayed through the
REFERENCE merge-tree (oracle/tsref/replay_ref.js, this container only), then
SnapshotV1.extractSync() + emit() (packages/dds/merge-tree/src/snapshotV1.ts:85-246); the
emitted tree entries (path -> parsed contents) are stored as <name>.snapshot.jsonl.
Fixtures are data only (reference outputs)."""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
SETS = ['scenarios', 'synth_c1', 'synth_c3', 'synth_c4', 'synth_tiny', 'markers', 'synth_markers']
CHUNKED = {'synth_c3': 300}   # a small mergeTreeSnapshotChunkSize: multi-chunk (header + body_i) trees


def main():
    subprocess.check_call([sys.executable, os.path.join(REPO, 'oracle/tsref/build_ref.py')])
    replay = os.path.join(REPO, 'oracle/tsref/replay_ref.js')
    for name in SETS:
        res = subprocess.run(['node', replay, 'snapshot', os.path.join(HERE, name + '.mtlog')], check=True,
                             capture_output=True, text=True)
        with open(os.path.join(HERE, name + '.snapshot.jsonl'), 'w') as f:
            f.write(res.stdout)
        print(name, os.path.getsize(os.path.join(HERE, name + '.snapshot.jsonl')), 'B')
    for name, chunk in CHUNKED.items():
        log = os.path.join(HERE, name + '.mtlog')
        res = subprocess.run(['node', replay, 'snapshot', log, '0', '1000000', str(chunk)], check=True,
                             capture_output=True, text=True)
        out = os.path.join(HERE, f'{name}.snapshot{chunk}.jsonl')
        with open(out, 'w') as f:
            f.write(res.stdout)
        print(os.path.basename(out), os.path.getsize(out), 'B')


if __name__ == '__main__':
    main()
