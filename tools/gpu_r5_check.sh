#!/bin/bash
# GPU check after a change: the -m gpu suite, smoke(), then the default bench line (C3 with its side
# lines) without the CPU baseline
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r5c
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r5c/tests.log 2>&1 || { tail -40 gpurun_out/r5c/tests.log; exit 1; }
tail -3 gpurun_out/r5c/tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5c/smoke.log 2>&1 || { tail -20 gpurun_out/r5c/smoke.log; exit 1; }
tail -1 gpurun_out/r5c/smoke.log
if [ -z "$NO_BENCH" ]; then
  timeout -k 10 500 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/r5c/bench_c3.json 2> gpurun_out/r5c/bench_c3.err || { tail -20 gpurun_out/r5c/bench_c3.err; exit 1; }
  python3 - <<'PY'
import json
d = json.loads(open('gpurun_out/r5c/bench_c3.json').read().strip().splitlines()[-1])
print('C3', round(d['value'] / 1e6, 1), 'M ops/s')
for k, v in d.get('slow_paths', {}).items():
    if isinstance(v, dict):
        print(k, v.get('value'), v.get('unit'), v['roofline'].get('kernel'), v['roofline'].get('avg_launch_ms'), v.get('parity'))
PY
fi
