#!/bin/bash
# Round-5 evidence on the GPU box at HEAD: smoke, the kernel trace + HBM passes (C3 with its side
# lines, C4, C5) copied to profiles/r05_pmc_traffic_<config>.json (bench.py reads them), the SQ
# counter passes of C3, then the default bench lines (C3 with side lines, C4, C5).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r5f
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5f/smoke.log 2>&1 || { tail -20 gpurun_out/r5f/smoke.log; exit 1; }
tail -1 gpurun_out/r5f/smoke.log
if [ -n "$PRE_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest $PRE_TESTS -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/r5f/pre_tests.log 2>&1 || { tail -30 gpurun_out/r5f/pre_tests.log; exit 1; }
  tail -1 gpurun_out/r5f/pre_tests.log
fi
for c in ${PROF_CONFIGS:-C3 C4 C5}; do
  S=; [ $c = C3 ] && S=1
  SLOW=$S CONFIG=$c bash tools/rocprof.sh > gpurun_out/r5f/rp_$c.log 2>&1 || { tail -20 gpurun_out/r5f/rp_$c.log; exit 1; }
  cp gpurun_out/rp_$c/pmc_traffic.json profiles/r05_pmc_traffic_$c.json || exit 1
  for f in pmc_traffic.json kernel_stats.csv tick_gaps.txt kt_bench.log; do cp gpurun_out/rp_$c/$f gpurun_out/r5f/${c}_$f || exit 1; done
  rm -rf gpurun_out/rp_$c  # (the rocprof databases: too large to bring back)
  echo "profiled $c"
done
if [ -z "$NO_SQ" ]; then
  bash tools/sq_pass.sh > gpurun_out/r5f/sq.log 2>&1 || { tail -20 gpurun_out/r5f/sq.log; exit 1; }
  cp gpurun_out/sq/p1.txt gpurun_out/r5f/sq_C3_pass1.txt && cp gpurun_out/sq/p2.txt gpurun_out/r5f/sq_C3_pass2.txt || exit 1
  rm -rf gpurun_out/sq
  echo "sq done"
fi
STEPS="${BENCHES:-bench c4 c5}" bash tools/gpu_check.sh > gpurun_out/r5f/benches.log 2>&1 || { tail -20 gpurun_out/r5f/benches.log; exit 1; }
cp gpurun_out/bench_c3.json gpurun_out/bench_c4.json gpurun_out/bench_c5.json gpurun_out/r5f/ || exit 1
cat gpurun_out/r5f/benches.log | cut -c1-600
echo evidence done
