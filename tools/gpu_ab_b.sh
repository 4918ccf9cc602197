#!/bin/bash
# Launch-size (b, ops per document per launch) A/B on the GPU box: the headline bench of C3 / C4 / C5
# at b = 32 and larger b, interleaved (rounds of every variant), without the side lines, H2D line or
# cpu baseline.  One JSON line per run in gpurun_out/ab_b_<config>.log.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
for r in 1 2; do
    for c in ${CONFIGS:-C5 C4 C3}; do
        case $c in
            C5) BS="32 64 128" ;;
            *) BS="32 48 64" ;;
        esac
        for b in $BS; do
            echo "round $r config $c b $b" >> gpurun_out/ab_b_$c.log
            timeout -k 10 240 python bench.py --config $c --ops-per-launch $b --steps 3 --warmup 1 --no-cpu-baseline \
                --no-slow-paths >> gpurun_out/ab_b_$c.log 2>> gpurun_out/ab_b.err || exit 1
        done
    done
done
