#!/bin/bash
# round 3, session 3: refresh the AR log_prob and Bayesian-MAF lines on the final tree
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/rf_$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/rf_$name.log | head -1)"
  if [ $rc -ne 0 ]; then tail -n 5 "gpurun_out/rf_$name.log"; exit $rc; fi
}
step nsa16 300 python bench.py --flow nsa16 --no-cpu-baseline
step maf 300 python bench.py --flow maf --no-cpu-baseline
step nsa 300 python bench.py --flow nsa --no-cpu-baseline
step nsa_sample 300 python bench.py --flow nsa --sample --no-cpu-baseline
step bayes_lp 300 python bench.py --bayes lp --no-cpu-baseline
step bayes_sample 300 python bench.py --bayes sample --no-cpu-baseline
exit 0
