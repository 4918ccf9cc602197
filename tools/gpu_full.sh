set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
STEPS="tests bench c4 c5" bash tools/gpu_check.sh || exit 1
timeout -k 10 300 python -u tools/bench_snapshot.py > gpurun_out/snapshot_bench.json 2> gpurun_out/snapshot_bench.err || { tail -20 gpurun_out/snapshot_bench.err; exit 1; }
cat gpurun_out/snapshot_bench.json
CONFIG=C3 bash tools/rocprof.sh || exit 1
CONFIG=C4 bash tools/rocprof.sh || exit 1
ls gpurun_out/rp_C3 gpurun_out/rp_C4
