#!/bin/bash
# One rocprofv3 PMC pass of SQ counters over a 1-step bench (run on the GPU box from the repo root).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/sq
mkdir -p $OUT
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_INSTS_LDS -d $OUT/p1 -o p1 -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-slow-paths > $OUT/p1.log 2>&1 || exit 1
timeout -s KILL 240 rocprofv3 --pmc SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_ANY SQ_INSTS_SMEM SQ_INSTS_VMEM GRBM_GUI_ACTIVE -d $OUT/p2 -o p2 -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-slow-paths > $OUT/p2.log 2>&1 || exit 1
python3 tools/rocpd_summary.py $OUT/p1/p1_results.db --pmc > $OUT/p1.txt && python3 tools/rocpd_summary.py $OUT/p2/p2_results.db --pmc > $OUT/p2.txt
