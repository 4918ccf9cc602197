#!/bin/bash
# GPU box: HBM-counter calibration (tools/pmc_calib.py) -- one rocprofv3 pass per counter group, then
# the same request-level counters over one C5 bench step (the kernel whose traffic they explain)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/calib
mkdir -p $OUT
timeout -s KILL 60 rocprofv3 -L > $OUT/avail.txt 2>&1 || true
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o fetch -- python3 tools/pmc_calib.py > $OUT/known.json 2> $OUT/fetch.err || { tail -5 $OUT/fetch.err; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o write -- python3 tools/pmc_calib.py > /dev/null 2> $OUT/write.err || { tail -5 $OUT/write.err; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum -d $OUT/req -o req -- python3 tools/pmc_calib.py > /dev/null 2> $OUT/req.err || { tail -5 $OUT/req.err; exit 1; }
python3 tools/pmc_traffic.py $OUT/fetch/fetch_results.db $OUT/write/write_results.db $OUT/traffic.json || exit 1
python3 tools/rocpd_summary.py $OUT/req/req_results.db --pmc > $OUT/req.txt || exit 1
cat $OUT/known.json; cat $OUT/req.txt | cut -c1-220
if [ -n "$BENCH_CONFIG" ]; then
  MTGPU_SERIAL=1 timeout -s KILL 240 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum -d $OUT/breq -o breq -- python3 bench.py --config $BENCH_CONFIG --steps 1 --warmup 0 --no-cpu-baseline --no-slow-paths > $OUT/breq.log 2>&1 || { tail -5 $OUT/breq.log; exit 1; }
  python3 tools/rocpd_summary.py $OUT/breq/breq_results.db --pmc > $OUT/breq.txt || exit 1
  grep -E "reg_apply|Kernel|kernel" $OUT/breq.txt | head -20 | cut -c1-220
fi
