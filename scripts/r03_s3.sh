#!/bin/bash
# round 3, session 3: ring-barrier wait placement A/B (ctx preloaded before the stage-A barrier;
# s_waitcnt builtin) and the parity subset
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
  local name=$1 t=$2; shift 2
  echo "=== $name" | tee -a gpurun_out/s3_steps.log
  timeout -k 10 "$t" "$@" > "gpurun_out/s3_$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a gpurun_out/s3_steps.log
  tail -n 8 "gpurun_out/s3_$name.log" | cut -c1-400
  if [ $rc -ne 0 ]; then exit $rc; fi
}
step parity 300 python -u -m pytest -m gpu -x -q --timeout 150 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_train.py
VARIANTS="base nowait glds" step ab 400 bash scripts/ab.sh
exit 0
