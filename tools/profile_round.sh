#!/bin/bash
# The round's rocprofv3 evidence on the GPU box (run from the repo root): for each config, a kernel
# trace + stats of the bench command with the classes serialized and its tick gaps, then the HBM PMC
# passes (tools/rocprof.sh); for C3 also the two SQ-counter passes (tools/sq_pass.sh).  Outputs land
# under gpurun_out/ (copied into profiles/ by hand, named per round).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
for cfg in ${CONFIGS:-C3 C4 C5}; do
  CONFIG=$cfg bash tools/rocprof.sh || { echo "rocprof $cfg failed"; exit 1; }
  echo "== $cfg"; head -4 gpurun_out/rp_$cfg/kernel_stats.csv | cut -c1-160; cat gpurun_out/rp_$cfg/tick_gaps.txt
done
if [ -z "$NO_SQ" ]; then
  bash tools/sq_pass.sh || { echo "sq pass failed"; exit 1; }
  echo "== SQ"; grep -A8 "reg_apply_kernelILi9E" gpurun_out/sq/p1.txt | head -9
fi
