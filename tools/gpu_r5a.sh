#!/bin/bash
# round 5: tick-major host-fed feed -- GPU tests of the new path, then driver-style bench lines
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/r5a
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py::test_tick_feed_equals_reference tests/test_gpu_parity.py::test_tick_feed_stops_at_a_malformed_tick tests/test_gpu_deli.py tests/test_positions.py > gpurun_out/r5a/tests.log 2>&1 || { tail -30 gpurun_out/r5a/tests.log; exit 1; }
tail -3 gpurun_out/r5a/tests.log
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-slow-paths --no-cpu-baseline > gpurun_out/r5a/c3.json 2> gpurun_out/r5a/c3.err || { tail -20 gpurun_out/r5a/c3.err; exit 1; }
timeout -k 10 300 python -u bench.py --config C5 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/r5a/c5.json 2> gpurun_out/r5a/c5.err || { tail -20 gpurun_out/r5a/c5.err; exit 1; }
timeout -k 10 300 python -u bench.py --config C4 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/r5a/c4.json 2> gpurun_out/r5a/c4.err || { tail -20 gpurun_out/r5a/c4.err; exit 1; }
for c in c3 c4 c5; do python3 -c "
import json,sys; d=json.load(open('gpurun_out/r5a/$c.json'))
print('$c', d['value'], d['value_hbm_resident']['value'], d['ms_per_step'], d['upload'])"; done
