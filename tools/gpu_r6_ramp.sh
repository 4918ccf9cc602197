#!/bin/bash
# A/B of the host-fed feed's first tick (bench.py --first-tick) on C5 and C3, interleaved, each run
# a fresh bench process (run on the GPU box from the repo root)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/ramp
mkdir -p $OUT
for rep in 1 2; do
  for cfg in C5 C3; do
    for ft in 0 8 2; do
      timeout -k 10 300 python3 bench.py --config $cfg --steps 3 --warmup 1 --no-cpu-baseline --no-slow-paths --first-tick $ft > $OUT/${cfg}_ft${ft}_$rep.json 2> $OUT/${cfg}_ft${ft}_$rep.err || { tail -20 $OUT/${cfg}_ft${ft}_$rep.err; exit 1; }
      python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], round(d['value']/1e6,2), round(d['value_hbm_resident']['value']/1e6,2))" $OUT/${cfg}_ft${ft}_$rep.json
    done
  done
done
