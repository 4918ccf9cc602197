set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/rp
timeout -k 10 120 rocprofv3 --list-avail > gpurun_out/rp/avail.txt 2>&1 || true
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/rp/kt -o kt -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/rp/kt_bench.log 2>&1
echo KT_EXIT $? >> gpurun_out/rp/kt_bench.log
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SMEM SQ_INSTS_VMEM -d gpurun_out/rp/pmc1 -o pmc1 -- python3 bench.py --docs 20000 --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/rp/pmc1.log 2>&1
echo PMC1_EXIT $? >> gpurun_out/rp/pmc1.log
