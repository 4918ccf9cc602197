#!/bin/bash
# SQ counters of the editing form on the farm (tools/farm_probe.py at b = 32): instructions and waits
# per record of mt::apply_kernel<256, false, true>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/farmsq
mkdir -p $OUT
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_INSTS_LDS -d $OUT/p1 -o p1 -- python3 tools/farm_probe.py 100000 32 > $OUT/p1.log 2>&1 || exit 1
timeout -s KILL 240 rocprofv3 --pmc SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_ANY SQ_INSTS_SMEM SQ_INSTS_VMEM GRBM_GUI_ACTIVE -d $OUT/p2 -o p2 -- python3 tools/farm_probe.py 100000 32 > $OUT/p2.log 2>&1 || exit 1
python3 tools/rocpd_summary.py $OUT/p1/p1_results.db --pmc > $OUT/p1.txt && python3 tools/rocpd_summary.py $OUT/p2/p2_results.db --pmc > $OUT/p2.txt || exit 1
rm -rf $OUT/p1 $OUT/p2
grep -A9 "apply_kernelILi256ELb0ELb1E" $OUT/p1.txt | head -20
grep -A9 "apply_kernelILi256ELb0ELb1E" $OUT/p2.txt | head -20
