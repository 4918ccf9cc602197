#!/bin/bash
# A/B of the class launch order (MTGPU_CLASS_ORDER=asc vs the default, largest capacity first) on
# C5, C4 and C3: fresh bench processes, interleaved (run on the GPU box from the repo root)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/order
mkdir -p $OUT
for rep in 1 2; do
  for cfg in C5 C4 C3; do
    for ord in asc desc; do
      MTGPU_CLASS_ORDER=$ord timeout -k 10 300 python3 bench.py --config $cfg --steps 3 --warmup 1 --no-cpu-baseline --no-slow-paths > $OUT/${cfg}_${ord}_$rep.json 2> $OUT/${cfg}_${ord}_$rep.err || { tail -20 $OUT/${cfg}_${ord}_$rep.err; exit 1; }
      python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], round(d['value']/1e6,2), round(d['value_hbm_resident']['value']/1e6,2), d['checksum_digest'])" $OUT/${cfg}_${ord}_$rep.json
    done
  done
done
