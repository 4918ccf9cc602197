#!/bin/bash
# Interleaved A/B of libmtgpu builds on the editing-client farm (tools/farm_probe.py, b = 32)
#   LIBS="fluidframework_amd/libmtgpu.so ablib/libmtgpu_locw3.so" tools/gpu_ab_farm.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/abfarm
for rep in 1 2; do
  for L in $LIBS; do
    MTGPU_LIB=$PWD/$L timeout -k 10 300 python3 -u tools/farm_probe.py 100000 32 > gpurun_out/abfarm/$(basename $L .so)_$rep.log 2>&1 || { tail -5 gpurun_out/abfarm/$(basename $L .so)_$rep.log; exit 1; }
    echo "$rep $L $(cut -c1-50 gpurun_out/abfarm/$(basename $L .so)_$rep.log | head -1) $(grep -o 'digest [0-9a-f]*' gpurun_out/abfarm/$(basename $L .so)_$rep.log)"
  done
done
