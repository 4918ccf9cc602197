set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
timeout -k 10 300 python -u tools/bench_positions.py > gpurun_out/positions.json 2> gpurun_out/positions.err || { tail -20 gpurun_out/positions.err; exit 1; }
cat gpurun_out/positions.json
timeout -k 10 900 python -u tools/ab.py --config C3 --reps 3 ablib/libmtgpu_base.so ablib/libmtgpu_new.so fluidframework_amd/libmtgpu.so > gpurun_out/ab_C3.log 2>&1 || { tail -20 gpurun_out/ab_C3.log; exit 1; }
tail -4 gpurun_out/ab_C3.log
