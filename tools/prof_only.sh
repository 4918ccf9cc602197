#!/bin/bash
# Per-phase cycles of the register engine, one phase per build (tools/build_variants.py with
# -DMT_PROF -DMT_PROF_ONLY=<slot>: one stamp pair per phase execution); run on the GPU box.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/prof
for lib in ablib/libmtgpu_p*.so; do
  n=$(basename $lib .so)
  MTGPU_LIB=$lib timeout -k 10 120 python3 -u tools/prof_phases.py --config ${CONFIG:-C3} --docs ${DOCS:-20000} > gpurun_out/prof/$n.log 2>&1 || { tail -5 gpurun_out/prof/$n.log; exit 1; }
  echo "== $n"; grep -E "^K= ?(6|9|10)" gpurun_out/prof/$n.log | cut -c1-200
done
