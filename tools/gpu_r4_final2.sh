#!/bin/bash
# Round-4 closing evidence on the GPU box after the small-class change: the -m gpu suite, smoke, the
# C5 kernel trace + HBM passes (its dominant kernel changed), then the default bench lines (C3 with
# side lines, C4, C5) reading that C5 PMC summary
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
CONFIG=C5 bash tools/rocprof.sh > gpurun_out/rp5.log 2>&1 || { tail -20 gpurun_out/rp5.log; exit 1; }
cp gpurun_out/rp_C5/pmc_traffic.json profiles/r04_pmc_traffic_C5.json
STEPS="bench c4 c5" bash tools/gpu_check.sh > gpurun_out/benches.log 2>&1 || { tail -20 gpurun_out/benches.log; exit 1; }
echo evidence done
