#!/bin/bash
# round 3, session 19: dim-grouped forward image (one dim per row quarter) — AR fused/maf parity
# tests, then the sampling and maf-gradient benches
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/s19_$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/s19_$name.log | head -1)" | tee -a gpurun_out/s19_steps.log
  tail -n 2 "gpurun_out/s19_$name.log" | cut -c1-300
  if [ $rc -ne 0 ]; then exit $rc; fi
}
step tests 600 python -u -m pytest tests/test_gpu_ar_fused.py tests/test_bayes_maf.py tests/test_gpu_train.py -x -q -m gpu --timeout 300 --timeout-method thread
step nsa16_sample 300 python bench.py --flow nsa16 --sample --no-cpu-baseline
step nsa_sample 300 python bench.py --flow nsa --sample --no-cpu-baseline
step maf_sample 300 python bench.py --flow maf --sample --no-cpu-baseline
step bayes_sample 300 python bench.py --bayes sample --no-cpu-baseline
step bayes_grad 300 python bench.py --bayes grad --no-cpu-baseline
exit 0
