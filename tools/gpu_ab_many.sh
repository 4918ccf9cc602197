#!/bin/bash
# GPU-box round trip: the -m gpu suite on the in-tree build (unless NO_TESTS), then an interleaved A/B
# of the libraries named in $LIBS on $CONFIG (default C3)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/gpu_tests.log 2>&1 || { tail -40 gpurun_out/gpu_tests.log; exit 1; }
  tail -2 gpurun_out/gpu_tests.log
fi
timeout -k 10 1000 python -u tools/ab.py --config ${CONFIG:-C3} --reps ${REPS:-3} ${LIBS} > gpurun_out/ab_${CONFIG:-C3}.log 2>&1 || { tail -20 gpurun_out/ab_${CONFIG:-C3}.log; exit 1; }
tail -8 gpurun_out/ab_${CONFIG:-C3}.log
