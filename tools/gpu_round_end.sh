#!/bin/bash
# Round-end rehearsal on the GPU box: the -m gpu suite, smoke(), the default bench line (C3 + side
# lines), C4 and C5 lines with their CPU baselines, an A/B of the previous build, one SQ pass.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
STEPS="tests" bash tools/gpu_check.sh || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
STEPS="bench c4 c5" bash tools/gpu_check.sh > gpurun_out/bench_lines.log 2>&1 || { tail -20 gpurun_out/bench_lines.log; exit 1; }
python3 -c "
import json
for c in ('c3', 'c4', 'c5'):
    d = json.load(open('gpurun_out/bench_%s.json' % c))
    cb = d.get('cpu_baseline') or {}
    print(c, d['value'], d['roofline']['kernel'], d['roofline']['frac'], (d.get('value_with_h2d') or {}).get('value'), cb.get('value'), cb.get('reference_estimate'), d.get('parity'))
"
if [ -f ablib/libmtgpu_prebin.so ]; then
  timeout -k 10 400 python3 -u tools/ab.py --reps 2 ablib/libmtgpu_prebin.so fluidframework_amd/libmtgpu.so > gpurun_out/ab_bin.log 2>&1 || exit 1
  grep -E "median|digest" gpurun_out/ab_bin.log
fi
bash tools/sq_pass.sh || exit 1
