#!/bin/bash
# round 3, session 4: the wide (H = 512 x 5) fused MAF sampler — tests, bench lines, trace
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
  local name=$1 t=$2; shift 2
  echo "=== $name" | tee -a gpurun_out/s4_steps.log
  timeout -k 10 "$t" "$@" > "gpurun_out/s4_$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a gpurun_out/s4_steps.log
  tail -n 6 "gpurun_out/s4_$name.log" | cut -c1-600
  if [ $rc -ne 0 ]; then exit $rc; fi
}
step tests 600 python -u -m pytest -m gpu -x -q --timeout 300 --timeout-method thread tests/test_gpu_ar_fused.py tests/test_gpu_parity.py
step maf4s 400 python bench.py --flow maf4 --sample --steps 10 --warmup 3
step maf4lp 600 python bench.py --flow maf4 --steps 3 --warmup 1
step bayes4 400 python bench.py --bayes sample --bayes-shape maf4 --steps 5 --warmup 2
step prof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_s4 -o run --output-format csv -- python3 bench.py --flow maf4 --sample --steps 5 --warmup 2 --no-cpu-baseline
exit 0
