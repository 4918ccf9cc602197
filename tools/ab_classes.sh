#!/bin/bash
# GPU-box A/B of libmtgpu builds (tools/ab.py) on several configs, after the -m gpu suite:
#   LIBS="ablib/a.so ablib/b.so" CONFIGS="C3 C4" REPS=2 TESTS=1 bash tools/ab_classes.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/gpu_tests_ab.log 2>&1 || { tail -30 gpurun_out/gpu_tests_ab.log; exit 1; }
  tail -2 gpurun_out/gpu_tests_ab.log
fi
for c in ${CONFIGS:-C3 C4}; do
  timeout -k 10 900 python -u tools/ab.py --config $c --reps ${REPS:-2} ${LIBS} > gpurun_out/ab_$c.log 2>&1 || { tail -20 gpurun_out/ab_$c.log; exit 1; }
  tail -$(( $(echo $LIBS | wc -w) + 1 )) gpurun_out/ab_$c.log
done
