#!/bin/bash
# Timeline of C5's host-fed steps (run on the GPU box from the repo root): kernel + memory-copy trace of
# one timed step, the host's per-tick split (MTGPU_TICK_TRACE=1) and tools/tick_timeline.py's view.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/c5tl
mkdir -p $OUT
MTGPU_TICK_TRACE=1 timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d $OUT/tr -o tr -- python3 bench.py --config C5 --steps 1 --warmup 1 --no-cpu-baseline --no-slow-paths > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 1; }
python3 tools/tick_timeline.py $OUT/tr/tr_results.db --min-mb 16 --events 700 --from-kernel restore_all --nth 2 > $OUT/timeline.txt || exit 1
python3 tools/tick_gaps.py $OUT/tr/tr_results.db > $OUT/tick_gaps.txt || exit 1
rm -rf $OUT/tr
grep -A1 mt_submit_ticks $OUT/bench.log | tail -6
grep -c . $OUT/timeline.txt; tail -4 $OUT/timeline.txt
