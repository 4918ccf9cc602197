#!/bin/bash
# C5 host-fed step under a kernel + memory-copy trace: where the 35 ms beyond the HBM-resident step go
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r5c
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d gpurun_out/r5c/tr -o tr -- python3 bench.py --config C5 --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/r5c/c5.json 2> gpurun_out/r5c/c5.err || { tail -20 gpurun_out/r5c/c5.err; exit 1; }
db=$(ls gpurun_out/r5c/tr/*.db gpurun_out/r5c/tr/*/*.db 2>/dev/null | head -1)
echo "db: $db"
python3 tools/tick_timeline.py "$db" --events 300 > gpurun_out/r5c/timeline.txt 2>&1
tail -5 gpurun_out/r5c/timeline.txt
rm -f "$db"
