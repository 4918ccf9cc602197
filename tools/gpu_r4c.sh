#!/bin/bash
# GPU box: events line A/B (HEAD build vs in-tree), C5 request counters with the scratch-free K = 4
# build, SQ counter passes and the kernel trace + HBM passes of C3 on the in-tree build
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/ev gpurun_out/calib
for lib in ablib/libmtgpu_head.so fluidframework_amd/libmtgpu.so; do
  MTGPU_LIB=$(pwd)/$lib timeout -k 10 300 python3 -u tools/bench_events.py >> gpurun_out/ev/bench_events.jsonl 2> gpurun_out/ev/err.log || { tail -20 gpurun_out/ev/err.log; exit 1; }
done
cut -c1-400 gpurun_out/ev/bench_events.jsonl
MTGPU_LIB=$(pwd)/ablib/libmtgpu_k4w4.so MTGPU_SERIAL=1 timeout -s KILL 240 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum -d gpurun_out/calib/breq4 -o breq4 -- python3 bench.py --config C5 --steps 1 --warmup 0 --no-cpu-baseline --no-slow-paths > gpurun_out/calib/breq4.log 2>&1 || { tail -5 gpurun_out/calib/breq4.log; exit 1; }
python3 tools/rocpd_summary.py gpurun_out/calib/breq4/breq4_results.db --pmc > gpurun_out/calib/breq4.txt || exit 1
grep -A4 "reg_apply_kernelILi4E" gpurun_out/calib/breq4.txt | tail -5
bash tools/sq_pass.sh > gpurun_out/sq.log 2>&1 || { tail -20 gpurun_out/sq.log; exit 1; }
CONFIG=C3 bash tools/rocprof.sh > gpurun_out/rp.log 2>&1 || { tail -20 gpurun_out/rp.log; exit 1; }
echo done
