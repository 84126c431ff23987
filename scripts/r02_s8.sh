#!/bin/bash
# unique-index gathers in the training walk: gradient tests, NUTS gradient line A/B (sort vs scatter)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -v --timeout 150 --timeout-method thread -m gpu \
  tests/test_gpu_grad.py tests/test_bayes_maf.py tests/test_gpu_ar_schedule.py > gpurun_out/s8_tests.log 2>&1 || { tail -40 gpurun_out/s8_tests.log; exit 1; }
tail -3 gpurun_out/s8_tests.log
timeout -k 10 300 python bench.py --bayes grad > gpurun_out/s8_grad.log 2>&1 || { tail -20 gpurun_out/s8_grad.log; exit 1; }
NAZ_GATHER_SORT=1 timeout -k 10 300 python bench.py --bayes grad --no-cpu-baseline > gpurun_out/s8_grad_sort.log 2>&1 || { tail -20 gpurun_out/s8_grad_sort.log; exit 1; }
for f in s8_grad s8_grad_sort; do python -c "import json,sys; r=json.loads(open('gpurun_out/$f.log').read().strip().splitlines()[-1]); print('$f', r['ms_per_step'], r['value'])"; done
