#!/bin/bash
# Round-4 evidence on the GPU box: smoke, the default bench lines (C3 with side lines, C4, C5), the
# SQ counter passes of C3, and the kernel trace + HBM passes (C3 with its side lines, C4, C5)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -2 gpurun_out/smoke.log
STEPS="bench c4 c5" bash tools/gpu_check.sh > gpurun_out/benches.log 2>&1 || { tail -20 gpurun_out/benches.log; exit 1; }
bash tools/sq_pass.sh > gpurun_out/sq.log 2>&1 || { tail -20 gpurun_out/sq.log; exit 1; }
SLOW=1 CONFIG=C3 bash tools/rocprof.sh > gpurun_out/rp3.log 2>&1 || { tail -20 gpurun_out/rp3.log; exit 1; }
CONFIG=C4 bash tools/rocprof.sh > gpurun_out/rp4.log 2>&1 || { tail -20 gpurun_out/rp4.log; exit 1; }
CONFIG=C5 bash tools/rocprof.sh > gpurun_out/rp5.log 2>&1 || { tail -20 gpurun_out/rp5.log; exit 1; }
echo evidence done
