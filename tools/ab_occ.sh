#!/bin/bash
# Occupancy A/B for the register classes (ablib/ variants from tools/build_variants.py, MT_WPE_OV /
# MT_WPE_C64_OV), interleaved.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python3 -u tools/ab.py --config C3W --reps 2 ablib/libmtgpu_base.so ablib/libmtgpu_c64a.so ablib/libmtgpu_c64b.so ablib/libmtgpu_c64c.so > gpurun_out/abocc_c3w.log 2>&1 || { tail -20 gpurun_out/abocc_c3w.log; exit 1; }
grep -E "median|rep" gpurun_out/abocc_c3w.log | cut -c1-400
