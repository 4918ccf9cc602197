#!/bin/bash
# Occupancy A/B of the side paths' kernels (run on the GPU box from the repo root): the C64 form on
# C3W through tools/ab.py, and the event kernels through bench.py's C3_events side line, one fresh
# bench process per library, interleaved.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/sideocc
mkdir -p $OUT
if [ -n "${C64_LIBS-ablib/libmtgpu_hd.so ablib/libmtgpu_c64a.so ablib/libmtgpu_c64b.so}" ]; then
  timeout -k 10 600 python3 -u tools/ab.py --config C3W --reps 2 ${C64_LIBS-ablib/libmtgpu_hd.so ablib/libmtgpu_c64a.so ablib/libmtgpu_c64b.so} > $OUT/c3w.log 2>&1 || { tail -20 $OUT/c3w.log; exit 1; }
  grep median $OUT/c3w.log
fi
for rep in 1 2; do
  for v in ${EV_VARIANTS:-hd ev8 ev8910}; do
    MTGPU_LIB=$PWD/ablib/libmtgpu_$v.so timeout -k 10 300 python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline > $OUT/ev_${v}_$rep.json 2> $OUT/ev_${v}_$rep.err || { tail -20 $OUT/ev_${v}_$rep.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1]))['slow_paths']['C3_events']; print(sys.argv[1], round(d['value']/1e6,2), d['roofline']['class_ms_serialized'], d['parity'])" $OUT/ev_${v}_$rep.json
  done
done
