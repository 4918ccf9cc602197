#!/bin/bash
# Round-3 GPU check: the -m gpu suite on the in-tree build, A/Bs of the register-engine variants
# (ablib/, tools/build_variants.py) on C3 / C4 / C5, then the default bench line (with its
# slow-path side lines).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/gpu_tests_r3.log 2>&1 || { tail -30 gpurun_out/gpu_tests_r3.log; exit 1; }
tail -2 gpurun_out/gpu_tests_r3.log
timeout -k 10 400 python3 -u tools/ab.py --reps 1 ablib/libmtgpu_head.so ablib/libmtgpu_fin.so ablib/libmtgpu_nohtop.so ablib/libmtgpu_nonlq.so > gpurun_out/ab5_c3.log 2>&1 || exit 1
grep -E "median|digest" gpurun_out/ab5_c3.log
timeout -k 10 300 python3 -u tools/ab.py --config C4 --reps 1 ablib/libmtgpu_head.so ablib/libmtgpu_fin.so > gpurun_out/ab5_c4.log 2>&1 || exit 1
grep -E "median|digest" gpurun_out/ab5_c4.log
timeout -k 10 300 python3 -u tools/ab.py --config C5 --reps 1 ablib/libmtgpu_head.so ablib/libmtgpu_fin.so > gpurun_out/ab5_c5.log 2>&1 || exit 1
grep -E "median|digest" gpurun_out/ab5_c5.log
timeout -k 10 500 python3 -u bench.py > gpurun_out/bench_c3.json 2> gpurun_out/bench_c3.err || { tail -20 gpurun_out/bench_c3.err; exit 1; }
cat gpurun_out/bench_c3.json
