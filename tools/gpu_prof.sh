#!/bin/bash
# GPU-box phase profile: one -DMT_PROF -DMT_PROF_ONLY=<slot> build per phase (ablib/libmtgpu_p<slot>.so,
# tools/build_variants.py), each replaying $CONFIG (default C3) on $DOCS documents; then optionally an
# interleaved A/B ($AB="libA libB").
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
for lib in ablib/libmtgpu_p*.so; do
  n=$(basename $lib .so)
  MTGPU_LIB=$lib timeout -k 10 120 python3 -u tools/prof_phases.py --config ${CONFIG:-C3} --docs ${DOCS:-20000} > gpurun_out/prof/$n.log 2>&1 || { tail -5 gpurun_out/prof/$n.log; exit 1; }
  echo "== $n"; grep -E "^K= ?(6|9|10)" gpurun_out/prof/$n.log | cut -c1-160
done
if [ -n "$AB" ]; then
  timeout -k 10 900 python -u tools/ab.py --config ${CONFIG:-C3} --reps ${REPS:-3} $AB > gpurun_out/ab_${CONFIG:-C3}.log 2>&1 || { tail -20 gpurun_out/ab_${CONFIG:-C3}.log; exit 1; }
  cat gpurun_out/ab_${CONFIG:-C3}.log
fi
