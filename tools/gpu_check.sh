#!/bin/bash
# GPU-box check: the -m gpu suite, then the default bench line, then C5 (deli + apply) and the
# two-rank path.  Each GPU step has its own time limit; the chain stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
STEPS=${STEPS:-tests bench c5}
for s in $STEPS; do
  case $s in
    tests) timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/gpu_tests.log 2>&1 || { tail -40 gpurun_out/gpu_tests.log; exit 1; } ; tail -3 gpurun_out/gpu_tests.log ;;
    bench) timeout -k 10 400 python -u bench.py > gpurun_out/bench_c3.json 2> gpurun_out/bench_c3.err || { tail -20 gpurun_out/bench_c3.err; exit 1; } ; cat gpurun_out/bench_c3.json ;;
    c5) timeout -k 10 400 python -u bench.py --config C5 > gpurun_out/bench_c5.json 2> gpurun_out/bench_c5.err || { tail -20 gpurun_out/bench_c5.err; exit 1; } ; cat gpurun_out/bench_c5.json ;;
    c4) timeout -k 10 400 python -u bench.py --config C4 > gpurun_out/bench_c4.json 2> gpurun_out/bench_c4.err || { tail -20 gpurun_out/bench_c4.err; exit 1; } ; cat gpurun_out/bench_c4.json ;;
    prof) timeout -k 10 300 python -u tools/prof_phases.py --config ${PCONFIG:-C3} > gpurun_out/prof_${PCONFIG:-C3}.log 2>&1 || { tail -20 gpurun_out/prof_${PCONFIG:-C3}.log; exit 1; } ; cat gpurun_out/prof_${PCONFIG:-C3}.log ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
