#!/bin/bash
# GPU box: the -m gpu suite on the in-tree build, counter calibration + C5 request counters, then
# C3 / C5 / C4 A/Bs of the round's builds
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
timeout -k 10 900 python -u tools/ab.py --config C3 --reps 3 ablib/libmtgpu_head.so fluidframework_amd/libmtgpu.so > gpurun_out/ab_C3.log 2>&1 || { tail -20 gpurun_out/ab_C3.log; exit 1; }
tail -3 gpurun_out/ab_C3.log
BENCH_CONFIG=C5 bash tools/pmc_calib.sh > gpurun_out/calib.log 2>&1 || { tail -20 gpurun_out/calib.log; exit 1; }
tail -30 gpurun_out/calib.log | cut -c1-250
timeout -k 10 900 python -u tools/ab.py --config C5 --reps 3 ablib/libmtgpu_base.so ablib/libmtgpu_head.so fluidframework_amd/libmtgpu.so ablib/libmtgpu_k4w4.so > gpurun_out/ab_C5.log 2>&1 || { tail -20 gpurun_out/ab_C5.log; exit 1; }
tail -5 gpurun_out/ab_C5.log
timeout -k 10 900 python -u tools/ab.py --config C4 --reps 3 ablib/libmtgpu_base.so ablib/libmtgpu_head.so fluidframework_amd/libmtgpu.so ablib/libmtgpu_k6w3.so > gpurun_out/ab_C4.log 2>&1 || { tail -20 gpurun_out/ab_C4.log; exit 1; }
tail -5 gpurun_out/ab_C4.log
