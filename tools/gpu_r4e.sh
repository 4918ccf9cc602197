#!/bin/bash
# GPU box: occupancy A/Bs of the side-line kernels -- C64 form on C3W (48 clients), event kernels on
# C3 with every callback recorded
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/ev
timeout -k 10 900 python -u tools/ab.py --config C3W --reps 2 fluidframework_amd/libmtgpu.so ablib/libmtgpu_c64w1.so ablib/libmtgpu_c64w1b.so > gpurun_out/ab_C3W.log 2>&1 || { tail -20 gpurun_out/ab_C3W.log; exit 1; }
tail -4 gpurun_out/ab_C3W.log
rm -f gpurun_out/ev/bench_events2.jsonl
for lib in fluidframework_amd/libmtgpu.so ablib/libmtgpu_ev1.so fluidframework_amd/libmtgpu.so ablib/libmtgpu_ev1.so; do
  MTGPU_LIB=$(pwd)/$lib timeout -k 10 300 python3 -u tools/bench_events.py >> gpurun_out/ev/bench_events2.jsonl 2> gpurun_out/ev/err.log || { tail -20 gpurun_out/ev/err.log; exit 1; }
done
cut -c1-200 gpurun_out/ev/bench_events2.jsonl
