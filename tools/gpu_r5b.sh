#!/bin/bash
# C5 host-fed pipeline: where the time goes (host checks vs apply loop), with and without tickets back
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/r5b
export MTGPU_TICK_TRACE=1
timeout -k 10 300 python -u bench.py --config C5 --steps 4 --warmup 1 --no-cpu-baseline > gpurun_out/r5b/c5.json 2> gpurun_out/r5b/c5.err || { tail -20 gpurun_out/r5b/c5.err; exit 1; }
timeout -k 10 300 python -u bench.py --config C5 --steps 4 --warmup 1 --no-cpu-baseline --no-tickets > gpurun_out/r5b/c5nt.json 2> gpurun_out/r5b/c5nt.err || { tail -20 gpurun_out/r5b/c5nt.err; exit 1; }
for c in c5 c5nt; do grep mt_submit_ticks gpurun_out/r5b/$c.err | tail -4; python3 -c "
import json,sys; d=json.load(open('gpurun_out/r5b/$c.json'))
print('$c', d['value'], d['value_hbm_resident']['value'], d['ms_per_step'])"; done
