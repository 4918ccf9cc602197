#!/bin/bash
# Interleaved A/B of libmtgpu builds (HBM-resident bench value) plus, per build, the two PMC passes
# (FETCH_SIZE, WRITE_SIZE) of the same config with the classes serialized: per-class traffic ratios.
#   CONFIGS="C5 C4" LIBS="ablib/libmtgpu_base.so ablib/libmtgpu_occB.so" tools/gpu_ab_pmc.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/abpmc
mkdir -p $OUT
for cfg in ${CONFIGS:-C5}; do
  timeout -k 10 900 python -u tools/ab.py --config $cfg --reps ${REPS:-2} --steps ${STEPS:-3} $LIBS > $OUT/ab_$cfg.log 2>&1 || { tail -20 $OUT/ab_$cfg.log; exit 1; }
  tail -4 $OUT/ab_$cfg.log
  if [ -z "$NO_PMC" ]; then
  for lib in $LIBS; do
    n=$(basename $lib .so)
    for c in FETCH_SIZE WRITE_SIZE; do
      MTGPU_LIB=$PWD/$lib MTGPU_SERIAL=1 timeout -s KILL 300 rocprofv3 --pmc $c -d $OUT/${cfg}_${n}_$c -o p -- python3 bench.py --config $cfg --steps 1 --warmup 0 --no-cpu-baseline --no-slow-paths --hbm-only > $OUT/${cfg}_${n}_$c.json 2> $OUT/${cfg}_${n}_$c.err || { tail -5 $OUT/${cfg}_${n}_$c.err; exit 1; }
    done
    python3 tools/pmc_traffic.py $OUT/${cfg}_${n}_FETCH_SIZE/p_results.db $OUT/${cfg}_${n}_WRITE_SIZE/p_results.db $OUT/${cfg}_${n}_pmc.json || exit 1
    rm -rf $OUT/${cfg}_${n}_FETCH_SIZE $OUT/${cfg}_${n}_WRITE_SIZE
    echo "== $cfg $n"
    python3 tools/pmc_classes.py $OUT/${cfg}_${n}_FETCH_SIZE.json $OUT/${cfg}_${n}_pmc.json | tee $OUT/${cfg}_${n}_classes.txt
  done
  fi
done
