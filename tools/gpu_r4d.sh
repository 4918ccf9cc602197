#!/bin/bash
# GPU box: occupancy A/B on C3, then the round's rocprof evidence (C3 with side lines, C4, C5) and the
# default bench line
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u tools/ab.py --config C3 --reps 3 fluidframework_amd/libmtgpu.so ablib/libmtgpu_k10w2.so ablib/libmtgpu_k7w3.so > gpurun_out/ab_C3.log 2>&1 || { tail -20 gpurun_out/ab_C3.log; exit 1; }
tail -4 gpurun_out/ab_C3.log
SLOW=1 CONFIG=C3 bash tools/rocprof.sh > gpurun_out/rp3.log 2>&1 || { tail -20 gpurun_out/rp3.log; exit 1; }
CONFIG=C5 bash tools/rocprof.sh > gpurun_out/rp5.log 2>&1 || { tail -20 gpurun_out/rp5.log; exit 1; }
CONFIG=C4 bash tools/rocprof.sh > gpurun_out/rp4.log 2>&1 || { tail -20 gpurun_out/rp4.log; exit 1; }
echo profiles done
