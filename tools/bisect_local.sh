#!/bin/bash
# Editing-form throughput across commits (ablib/bisect/<commit>/: that commit's Python host, library
# and tools/bench_local.py), then the in-tree build; run on the GPU box.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
for d in ablib/bisect/*/ .; do
  (cd $d && timeout -k 10 200 python3 -u tools/bench_local.py --docs 8192 --reps 2 --cpu-docs 0 2>/dev/null | tail -1) > gpurun_out/bisect_$(basename $(realpath $d)).json || exit 1
  echo "$d $(python3 -c "import json,sys; d=json.load(open('gpurun_out/bisect_$(basename $(realpath $d)).json')); print(d['value'], d['best_s'])")"
done
