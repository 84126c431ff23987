#!/bin/bash
# round 3, session 6: bf16x6 weight-gradient kernel — gradient tests, then train / NUTS / CNF-train
# A/B against the fp32 wgrad_t16 (NAZ_WGRAD_X6=0) on the same box
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
  local name=$1 t=$2; shift 2
  echo "=== $name" | tee -a gpurun_out/s6_steps.log
  timeout -k 10 "$t" "$@" > "gpurun_out/s6_$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a gpurun_out/s6_steps.log
  tail -n 3 "gpurun_out/s6_$name.log" | cut -c1-300
  if [ $rc -ne 0 ]; then exit $rc; fi
}
step tests 600 python -u -m pytest -m gpu -x -q --timeout 300 --timeout-method thread tests/test_gpu_grad.py tests/test_gpu_train.py tests/test_bayes_maf.py tests/test_gpu_cnf_grad.py
step train_x6 400 python bench.py --train --steps 3 --warmup 1 --no-cpu-baseline
NAZ_WGRAD_X6=0 step train_t16 400 python bench.py --train --steps 3 --warmup 1 --no-cpu-baseline
step grad_x6 300 python bench.py --bayes grad --steps 10 --warmup 3 --no-cpu-baseline
NAZ_WGRAD_X6=0 step grad_t16 300 python bench.py --bayes grad --steps 10 --warmup 3 --no-cpu-baseline
step cnft_x6 400 python bench.py --cnf-train --steps 3 --warmup 1 --no-cpu-baseline
NAZ_WGRAD_X6=0 step cnft_t16 400 python bench.py --cnf-train --steps 3 --warmup 1 --no-cpu-baseline
step prof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_s6 -o run --output-format csv -- python3 bench.py --train --steps 2 --warmup 1 --no-cpu-baseline
exit 0
