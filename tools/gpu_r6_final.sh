#!/bin/bash
# Round-6 evidence on the GPU box at HEAD, in two calls (each within one gpurun limit):
#   PART=A: smoke, the kernel trace + HBM PMC passes of C3 (with its side lines), the SQ passes of C3;
#   PART=B: the kernel trace + HBM PMC passes of C4 and C5, then the driver-style bench lines
#           (C3 with its side lines and CPU baseline, C4, C5).
# Copies go to gpurun_out/r6f/ (profiles/r06_* are copied from there on the build host).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r6f
prof() {  # $1 = config, $2 = SLOW (1: the PMC passes include the side lines)
  SLOW=$2 CONFIG=$1 bash tools/rocprof.sh > gpurun_out/r6f/rp_$1.log 2>&1 || { tail -20 gpurun_out/r6f/rp_$1.log; return 1; }
  for f in pmc_traffic.json kernel_stats.csv tick_gaps.txt kt_bench.log; do cp gpurun_out/rp_$1/$f gpurun_out/r6f/${1}_$f || return 1; done
  cp gpurun_out/rp_$1/pmc_traffic.json profiles/r06_pmc_traffic_$1.json || return 1  # (bench.py PMC_ROUND: read below)
  rm -rf gpurun_out/rp_$1  # (the rocprof databases: too large to bring back)
  echo "profiled $1"
}
if [ "${PART:-A}" = A ]; then
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6f/smoke.log 2>&1 || { tail -20 gpurun_out/r6f/smoke.log; exit 1; }
  tail -1 gpurun_out/r6f/smoke.log
  prof C3 1 || exit 1
  bash tools/sq_pass.sh > gpurun_out/r6f/sq.log 2>&1 || { tail -20 gpurun_out/r6f/sq.log; exit 1; }
  cp gpurun_out/sq/p1.txt gpurun_out/r6f/sq_C3_pass1.txt && cp gpurun_out/sq/p2.txt gpurun_out/r6f/sq_C3_pass2.txt || exit 1
  cp gpurun_out/sq/p1.txt profiles/r06_sq_counters_C3_pass1.txt && cp gpurun_out/sq/p2.txt profiles/r06_sq_counters_C3_pass2.txt || exit 1
  rm -rf gpurun_out/sq
  echo "part A done"
else
  for c in ${PROF_CONFIGS:-C4 C5}; do prof $c "" || exit 1; done
  STEPS="${BENCHES:-bench c4 c5}" bash tools/gpu_check.sh > gpurun_out/r6f/benches.log 2>&1 || { tail -20 gpurun_out/r6f/benches.log; exit 1; }
  for f in bench_c3.json bench_c4.json bench_c5.json; do [ -f gpurun_out/$f ] && cp gpurun_out/$f gpurun_out/r6f/; done
  cut -c1-600 gpurun_out/r6f/benches.log
  echo "part B done"
fi
