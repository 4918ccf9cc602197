#!/usr/bin/env python3
"""A/B of libmtgpu builds on the GPU box: bench.py in a fresh process per run, variants interleaved
(A B A B ...) so clock / thermal drift hits both alike.  Prints per-variant median ops/s and the
dominant kernel's launch time.  Usage: tools/ab.py [--config C3] [--reps 3] ablib/libA.so ablib/libB.so"""
import argparse
import json
import os
import statistics
import subprocess
import sys

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ap = argparse.ArgumentParser()
ap.add_argument('libs', nargs='+')
ap.add_argument('--config', default='C3')
ap.add_argument('--reps', type=int, default=3)
ap.add_argument('--steps', type=int, default=2)
ap.add_argument('--docs', type=int, default=0)
a = ap.parse_args()
res = {lib: [] for lib in a.libs}
for r in range(a.reps):
    for lib in a.libs:
        env = dict(os.environ, MTGPU_LIB=os.path.abspath(lib))
        cmd = [sys.executable, os.path.join(HERE, 'bench.py'), '--no-cpu-baseline', '--no-slow-paths', '--hbm-only',
               '--config', a.config,
               '--steps', str(a.steps), '--warmup', '1'] + (['--docs', str(a.docs)] if a.docs else [])
        out = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300)
        if out.returncode:
            print(lib, 'FAILED', out.stderr[-1500:], flush=True)
            sys.exit(1)
        line = json.loads([x for x in out.stdout.split('\n') if x.startswith('{')][0])
        rf = line['roofline']
        res[lib].append((line['value'], rf['avg_launch_ms'], rf['kernel'], line['checksum_digest']))
        ak = rf.get('all_apply_kernels', {})
        print(f'rep {r} {os.path.basename(lib)}: {line["value"] / 1e6:.1f} M ops/s, {rf["kernel"]} '
              f'{rf["avg_launch_ms"]:.3f} ms, all apply kernels {ak.get("kernel_ms")} ms / {ak.get("launches")}, '
              f'classes {rf.get("class_ms_serialized")}, digest {line["checksum_digest"]}', flush=True)
for lib, v in res.items():
    print(f'{os.path.basename(lib)}: median {statistics.median(x[0] for x in v) / 1e6:.2f} M ops/s, '
          f'kernel {statistics.median(x[1] for x in v):.3f} ms')
digests = {x[3] for v in res.values() for x in v}
print('digests agree' if len(digests) == 1 else f'DIGESTS DIFFER {digests}')
