#!/bin/bash
# round 3, session 12: fused maf training path + refactored MafGrad
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
  local name=$1 t=$2; shift 2
  echo "=== $name" | tee -a gpurun_out/s12_steps.log
  timeout -k 10 "$t" "$@" > "gpurun_out/s12_$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a gpurun_out/s12_steps.log
  tail -n 30 "gpurun_out/s12_$name.log" | cut -c1-600
  if [ $rc -ne 0 ]; then exit $rc; fi
}
step tests 500 python -u -m pytest tests/test_bayes_maf.py tests/test_gpu_train.py -x -q -m gpu --timeout 200 --timeout-method thread -k "maf or lp_and_grad"
step bench 300 python bench.py --bayes grad --steps 10 --warmup 3
exit 0
