#!/bin/bash
# Round-3 check on the GPU box: the -m gpu suite, the editing-client farm, an A/B of one variant on C3,
# then the default bench line with its side lines.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/gpu_tests_r3b.log 2>&1 || { tail -30 gpurun_out/gpu_tests_r3b.log; exit 1; }
tail -2 gpurun_out/gpu_tests_r3b.log
timeout -k 10 200 python3 -u tools/bench_local.py --docs 8192 --reps 2 --cpu-docs 64 > gpurun_out/bench_local.json 2>/dev/null || exit 1
tail -1 gpurun_out/bench_local.json | cut -c1-250
timeout -k 10 400 python3 -u tools/ab.py --reps 1 fluidframework_amd/libmtgpu.so ablib/libmtgpu_k11w3.so > gpurun_out/ab_k11.log 2>&1 || exit 1
grep -E "median|digest" gpurun_out/ab_k11.log
timeout -k 10 600 python3 -u bench.py > gpurun_out/bench_c3.json 2> gpurun_out/bench_c3.err || { tail -20 gpurun_out/bench_c3.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/bench_c3.json')); print(d['value'], d['roofline']['kernel'], d['roofline']['frac']); [print(k, v['value'], v['unit'], v['roofline']['kernel'], v['parity']) for k, v in d['slow_paths'].items()]"
