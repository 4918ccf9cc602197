#!/bin/bash
# Round-6 GPU round trip: the -m gpu suite on the in-tree build, an interleaved C3 A/B of $BASE against
# it, then (unless NO_PROF) the per-phase profile over ablib/libmtgpu_p*.so and the SQ passes of the
# in-tree build (tools/gpu_r6_prof.sh).  Logs under gpurun_out/r6c/.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r6c
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/r6c/gpu_tests.log 2>&1 || { tail -40 gpurun_out/r6c/gpu_tests.log; exit 1; }
  tail -2 gpurun_out/r6c/gpu_tests.log
fi
if [ -n "$BASE" ]; then
  timeout -k 10 600 python -u tools/ab.py --config ${CONFIG:-C3} --reps ${REPS:-3} $BASE ${NEW:-fluidframework_amd/libmtgpu.so} > gpurun_out/r6c/ab_${CONFIG:-C3}.log 2>&1 || { tail -20 gpurun_out/r6c/ab_${CONFIG:-C3}.log; exit 1; }
  tail -3 gpurun_out/r6c/ab_${CONFIG:-C3}.log
fi
if [ -z "$NO_PROF" ]; then
  bash tools/gpu_r6_prof.sh > gpurun_out/r6c/prof.log 2>&1 || { tail -20 gpurun_out/r6c/prof.log; exit 1; }
  tail -40 gpurun_out/r6c/prof.log
fi
echo check done
