#!/bin/bash
# GPU-box round trip for a kernel change: the -m gpu suite on the in-tree build, then an interleaved
# A/B of ablib/libmtgpu_base.so (or $BASE) against the in-tree build (or $NEW) on $CONFIG (default C3).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/gpu_tests.log 2>&1 || { tail -40 gpurun_out/gpu_tests.log; exit 1; }
  tail -2 gpurun_out/gpu_tests.log
fi
timeout -k 10 900 python -u tools/ab.py --config ${CONFIG:-C3} --reps ${REPS:-3} ${BASE:-ablib/libmtgpu_base.so} ${NEW:-fluidframework_amd/libmtgpu.so} ${EXTRA} > gpurun_out/ab_${CONFIG:-C3}.log 2>&1 || { tail -20 gpurun_out/ab_${CONFIG:-C3}.log; exit 1; }
cat gpurun_out/ab_${CONFIG:-C3}.log
