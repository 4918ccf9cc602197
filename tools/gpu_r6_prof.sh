#!/bin/bash
# Round-6 attribution pass on the GPU box: per-phase cycles of the register engine (one MT_PROF_ONLY
# build per phase, tools/prof_only.sh over ablib/libmtgpu_p*.so) and the SQ counter passes of the
# in-tree build on C3 (tools/sq_pass.sh), copied to gpurun_out/r6prof/.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r6prof
bash tools/prof_only.sh > gpurun_out/r6prof/phases.log 2>&1 || { tail -20 gpurun_out/r6prof/phases.log; exit 1; }
cp gpurun_out/prof/*.log gpurun_out/r6prof/ || exit 1
if [ -z "$NO_SQ" ]; then
  bash tools/sq_pass.sh > gpurun_out/r6prof/sq.log 2>&1 || { tail -20 gpurun_out/r6prof/sq.log; exit 1; }
  cp gpurun_out/sq/p1.txt gpurun_out/r6prof/sq_C3_pass1.txt && cp gpurun_out/sq/p2.txt gpurun_out/r6prof/sq_C3_pass2.txt || exit 1
  rm -rf gpurun_out/sq
fi
cat gpurun_out/r6prof/phases.log
echo prof done
