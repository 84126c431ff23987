#!/bin/bash
# batched fused AR log-density: parity tests, bayes lp line + kernel trace
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 150 --timeout-method thread -m gpu \
  tests/test_gpu_ar_fused.py tests/test_bayes_maf.py > gpurun_out/s5_tests.log 2>&1 || { tail -40 gpurun_out/s5_tests.log; exit 1; }
tail -3 gpurun_out/s5_tests.log
timeout -k 10 300 python bench.py --bayes lp > gpurun_out/s5_lp.log 2>&1 || { tail -20 gpurun_out/s5_lp.log; exit 1; }
grep '^{' gpurun_out/s5_lp.log | cut -c1-600
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_s5 -o run --output-format csv -- python3 bench.py --bayes lp --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/s5_prof.log 2>&1 || { tail -20 gpurun_out/s5_prof.log; exit 1; }
head -6 gpurun_out/prof_s5/run_kernel_stats.csv | cut -c1-220
