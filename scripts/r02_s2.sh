#!/bin/bash
# round 2, session 2: fused AR (maf) + CNF gradient tests, then the maf / nsa flow lines
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -m gpu -x -v --timeout 150 --timeout-method thread \
  tests/test_gpu_ar_fused.py tests/test_gpu_cnf_grad.py tests/test_gpu_cnf.py > gpurun_out/s2_tests.log 2>&1
rc=$?
tail -40 gpurun_out/s2_tests.log
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
timeout -k 10 200 python bench.py --flow maf > gpurun_out/bench_maf.log 2>&1 || exit $?
timeout -k 10 200 python bench.py --flow nsa > gpurun_out/bench_nsa.log 2>&1 || exit $?
tail -2 gpurun_out/bench_maf.log gpurun_out/bench_nsa.log
exit $rc
