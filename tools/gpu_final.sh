#!/bin/bash
# Round-end rehearsal on the GPU box: the -m gpu suite, smoke(), the default bench line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
STEPS="tests" bash tools/gpu_check.sh || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
cat gpurun_out/smoke.log
STEPS="bench" bash tools/gpu_check.sh || exit 1
