#!/bin/bash
# one-context-vector pass-0 path: fused AR + bayes tests, maf_grid line A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 150 --timeout-method thread -m gpu \
  tests/test_gpu_ar_fused.py tests/test_bayes_maf.py tests/test_gpu_flow_abi.py > gpurun_out/s9_tests.log 2>&1 || { tail -40 gpurun_out/s9_tests.log; exit 1; }
tail -3 gpurun_out/s9_tests.log
timeout -k 10 300 python bench.py --flow maf_grid > gpurun_out/s9_grid.log 2>&1 || { tail -20 gpurun_out/s9_grid.log; exit 1; }
NAZ_AR_PASS0=0 timeout -k 10 300 python bench.py --flow maf_grid --no-cpu-baseline > gpurun_out/s9_grid0.log 2>&1 || { tail -20 gpurun_out/s9_grid0.log; exit 1; }
timeout -k 10 300 python bench.py --bayes lp --no-cpu-baseline > gpurun_out/s9_lp.log 2>&1 || { tail -20 gpurun_out/s9_lp.log; exit 1; }
for f in s9_grid s9_grid0 s9_lp; do python -c "import json,sys; r=json.loads(open('gpurun_out/$f.log').read().strip().splitlines()[-1]); print('$f', r['ms_per_step'], r['value'])"; done
