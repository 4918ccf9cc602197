#!/bin/bash
# Scheduler-strategy A/B of the register engine (ablib/ variants from tools/build_variants.py).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python3 -u tools/ab.py --config C3 --reps 2 ablib/libmtgpu_base.so ablib/libmtgpu_ilp.so ablib/libmtgpu_bias0.so ablib/libmtgpu_bias100.so > gpurun_out/absched_c3.log 2>&1 || { tail -20 gpurun_out/absched_c3.log; exit 1; }
grep -E "median" gpurun_out/absched_c3.log
timeout -k 10 400 python3 -u tools/ab.py --config C5 --reps 2 ablib/libmtgpu_base.so ablib/libmtgpu_ilp.so > gpurun_out/absched_c5.log 2>&1 || { tail -20 gpurun_out/absched_c5.log; exit 1; }
grep -E "median" gpurun_out/absched_c5.log
