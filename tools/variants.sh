#!/bin/bash
# A/B the in-tree libmtgpu.so against builds in fluidframework_amd/variants/ (bench.py lines only).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/var
for cfg in ${CONFIGS:-C3}; do
  for v in base ${VARIANTS}; do
    lib=""
    [ "$v" != base ] && lib=fluidframework_amd/variants/libmtgpu_$v.so
    MTGPU_LIB=$lib timeout -k 10 240 python3 -u bench.py --config $cfg --no-cpu-baseline > gpurun_out/var/${cfg}_$v.log 2>&1 || exit 1
    echo "$cfg $v $(tail -1 gpurun_out/var/${cfg}_$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["kernel"], d["parity"])')"
  done
done
