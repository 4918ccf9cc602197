#!/bin/bash
# The LDS-engine side paths on the GPU box: the -m gpu suite, the editing-client farm (tools/bench_local.py)
# and C3 with 48 clients (bench.py --config C3W) for the committed-HEAD library vs the in-tree one.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/gpu_tests_c64.log 2>&1 || { tail -30 gpurun_out/gpu_tests_c64.log; exit 1; }
tail -2 gpurun_out/gpu_tests_c64.log
for L in ablib/libmtgpu_head.so fluidframework_amd/libmtgpu.so; do
  MTGPU_LIB=$PWD/$L timeout -k 10 200 python3 -u tools/bench_local.py --docs 8192 --reps 2 --cpu-docs 0 > gpurun_out/local_$(basename $L .so).json 2>&1 || exit 1
  echo "$L $(tail -1 gpurun_out/local_$(basename $L .so).json | cut -c1-300)"
done
timeout -k 10 400 python3 -u tools/ab.py --config C3W --reps 1 ablib/libmtgpu_head.so fluidframework_amd/libmtgpu.so > gpurun_out/ab_c3w.log 2>&1 || exit 1
grep -E "median|digest" gpurun_out/ab_c3w.log
