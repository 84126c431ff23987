#!/bin/bash
# round 3, session 10: the fused maf backward (NUTS potential gradient): tests, bench line, kernel trace
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
  local name=$1 t=$2; shift 2
  echo "=== $name" | tee -a gpurun_out/s10_steps.log
  timeout -k 10 "$t" "$@" > "gpurun_out/s10_$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a gpurun_out/s10_steps.log
  tail -n 25 "gpurun_out/s10_$name.log" | cut -c1-600
  if [ $rc -ne 0 ]; then exit $rc; fi
}
step tests 400 python -u -m pytest tests/test_bayes_maf.py -x -v -m gpu --timeout 120 --timeout-method thread -k "fused_maf_backward or fused_full_size or lp_and_grad_vs_oracle"; step tests2 400 python -u -m pytest tests/test_gpu_grad.py -x -q -m gpu --timeout 120 --timeout-method thread -k "wgrad or gemm"
step bench 300 python bench.py --bayes grad --steps 10 --warmup 3 --no-cpu-baseline
step prof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_s10 -o run --output-format csv -- python bench.py --bayes grad --steps 10 --warmup 3 --no-cpu-baseline
exit 0
