#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/r5d
export MTGPU_TICK_TRACE=1
timeout -k 10 300 python -u bench.py --config C5 --steps 2 --warmup 1 --no-cpu-baseline --no-tickets > gpurun_out/r5d/c5.json 2> gpurun_out/r5d/c5.err || { tail -20 gpurun_out/r5d/c5.err; exit 1; }
timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-slow-paths > gpurun_out/r5d/c3.json 2> gpurun_out/r5d/c3.err || { tail -20 gpurun_out/r5d/c3.err; exit 1; }
grep mt_submit gpurun_out/r5d/*.err
