#!/bin/bash
# round 3, session 7: wgrad_x6 with two 4-wave workgroups per CU — gradient tests + train trace
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
  local name=$1 t=$2; shift 2
  echo "=== $name" | tee -a gpurun_out/s7_steps.log
  timeout -k 10 "$t" "$@" > "gpurun_out/s7_$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a gpurun_out/s7_steps.log
  tail -n 3 "gpurun_out/s7_$name.log" | cut -c1-300
  if [ $rc -ne 0 ]; then exit $rc; fi
}
step tests 600 python -u -m pytest -m gpu -x -q --timeout 300 --timeout-method thread tests/test_gpu_grad.py tests/test_gpu_train.py tests/test_gpu_cnf_grad.py
step train 400 python bench.py --train --steps 3 --warmup 1 --no-cpu-baseline
step prof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_s7 -o run --output-format csv -- python3 bench.py --train --steps 2 --warmup 1 --no-cpu-baseline
step cnft 400 python bench.py --cnf-train --steps 3 --warmup 1 --no-cpu-baseline
exit 0
