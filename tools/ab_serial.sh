#!/bin/bash
# A/B: capacity classes of a tick on concurrent streams (default) vs one after another.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/ab
for cfg in ${CONFIGS:-C3}; do
  for ser in 1 0; do
    MTGPU_SERIAL=$ser timeout -k 10 240 python3 -u bench.py --config $cfg --no-cpu-baseline > gpurun_out/ab/${cfg}_serial$ser.log 2>&1 || exit 1
    echo "$cfg serial=$ser $(tail -1 gpurun_out/ab/${cfg}_serial$ser.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(d["value"], r["kernel"], r["avg_launch_ms"], r["all_apply_kernels"])')"
  done
done
