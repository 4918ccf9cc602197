#!/usr/bin/env python3
"""Calibrate the GPU box's CPU baseline (js/observerReplay.js, a JavaScript restatement of the
observer apply path) against the reference itself (the type-stripped merge-tree in oracle/_tsref,
replayed by oracle/tsref/replay_ref.js), here in the build container, on identical logs with the
same worker_threads count: r = reference ops/s / restatement ops/s.  bench.py reports the
restatement's rate on the GPU box's cores and r x that rate as the reference estimate.

TEST / MEASUREMENT INFRASTRUCTURE ONLY (needs /root/reference + node).
Writes profiles/<round>_js_calibration.json."""
import argparse
import json
import os
import statistics
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)

from fluidframework_amd.oplog import CONFIGS  # noqa: E402
from oracle import oracle  # noqa: E402


def rate(cmd):
    out = subprocess.run(cmd, check=True, capture_output=True, text=True).stdout.strip().split('\n')[-1]
    r = json.loads(out)
    return r.get('apply_ops_per_sec') or r['ops_per_sec']


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--config', default='C3')
    ap.add_argument('--docs', type=int, default=1536)
    ap.add_argument('--threads', type=int, default=os.cpu_count())
    ap.add_argument('--reps', type=int, default=3)
    ap.add_argument('--out', default=None, help='default: profiles/r04_js_calibration_<config>[_t<threads>].json')
    a = ap.parse_args()
    subprocess.check_call([sys.executable, os.path.join(HERE, 'build_ref.py')], stdout=subprocess.DEVNULL)
    cfg = dict(CONFIGS[a.config])
    cfg.pop('n_docs')
    log = oracle.generate(a.docs, seed=20261015, **cfg)
    path = '/tmp/mtgpu_calibration.mtlog'
    log.save(path)
    ref, js = [], []
    for _ in range(a.reps):   # interleaved
        ref.append(rate(['node', os.path.join(HERE, 'replay_ref.js'), 'bench', path, str(a.threads)]))
        js.append(rate(['node', os.path.join(REPO, 'js', 'observerReplay.js'), 'bench', path, str(a.threads)]))
    res = {'config': a.config, 'docs': a.docs, 'ops': int(log.n_ops), 'threads': a.threads,
           'reference_ops_per_sec': statistics.median(ref), 'restatement_ops_per_sec': statistics.median(js),
           'r': statistics.median(ref) / statistics.median(js), 'reps': {'reference': ref, 'restatement': js},
           'how': 'apply-only rate (max over workers of time inside the apply loops), messages pre-built, '
                  'docs round-robin over worker_threads (replayMultipleFiles.ts:123-190 pattern)'}
    out = a.out or os.path.join(REPO, 'profiles', f'r04_js_calibration_{a.config}' +
                                ('' if a.threads == os.cpu_count() else f'_t{a.threads}') + '.json')
    with open(out, 'w') as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res))


if __name__ == '__main__':
    main()
