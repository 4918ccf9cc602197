#!/bin/bash
# the whole -m gpu suite on the in-tree build, then smoke()
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/r5t
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/r5t/tests.log 2>&1 || { tail -40 gpurun_out/r5t/tests.log; exit 1; }
tail -3 gpurun_out/r5t/tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5t/smoke.log 2>&1 || { tail -20 gpurun_out/r5t/smoke.log; exit 1; }
tail -1 gpurun_out/r5t/smoke.log
