#!/bin/bash
# rocprofv3 evidence for the round's bench (run on the GPU box from the repo root):
#   kernel trace + stats of the default bench command (classes serialized, MTGPU_SERIAL=1, so each
#   kernel's average duration is its own, as bench.py's roofline pass measures it), then one PMC pass per HBM counter
#   (FETCH_SIZE and WRITE_SIZE do not fit one pass: 3 + 2 TCC counters > 4).  SLOW=1: the PMC passes
#   include bench.py's side lines (their kernels have names of their own: events, C64, editing form).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
CONFIG=${CONFIG:-C3}
OUT=gpurun_out/rp_$CONFIG
mkdir -p $OUT
MTGPU_SERIAL=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt -o kt -- python3 bench.py --config $CONFIG --steps 2 --warmup 1 --no-cpu-baseline --no-slow-paths > $OUT/kt_bench.log 2>&1 || exit 1
SP=--no-slow-paths
[ -n "$SLOW" ] && SP=
MTGPU_SERIAL=1 timeout -s KILL 400 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o fetch -- python3 bench.py --config $CONFIG --steps 1 --warmup 0 --no-cpu-baseline $SP > $OUT/fetch.log 2>&1 || exit 1
MTGPU_SERIAL=1 timeout -s KILL 400 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o write -- python3 bench.py --config $CONFIG --steps 1 --warmup 0 --no-cpu-baseline $SP > $OUT/write.log 2>&1 || exit 1
python3 tools/rocpd_summary.py $OUT/kt/kt_results.db --csv $OUT/kernel_stats.csv || exit 1
python3 tools/pmc_traffic.py $OUT/fetch/fetch_results.db $OUT/write/write_results.db $OUT/pmc_traffic.json || exit 1
python3 tools/tick_gaps.py $OUT/kt/kt_results.db > $OUT/tick_gaps.txt || exit 1
