set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/gpu_tests_cls.log 2>&1 || { tail -30 gpurun_out/gpu_tests_cls.log; exit 1; }
tail -2 gpurun_out/gpu_tests_cls.log
timeout -k 10 900 python -u tools/ab.py --config C3 --reps 2 ablib/base.so ablib/cls.so ablib/cls_w6x4.so > gpurun_out/ab_cls_c3.log 2>&1 || { tail -20 gpurun_out/ab_cls_c3.log; exit 1; }
tail -4 gpurun_out/ab_cls_c3.log
timeout -k 10 900 python -u tools/ab.py --config C4 --reps 2 ablib/base.so ablib/cls.so ablib/cls_w6x4.so > gpurun_out/ab_cls_c4.log 2>&1 || { tail -20 gpurun_out/ab_cls_c4.log; exit 1; }
tail -4 gpurun_out/ab_cls_c4.log
