#!/bin/bash
# round-2 measurement set: smoke, GPU suite, headline bench + kernel trace, CNF-train line + trace,
# config-3 AR variant line.  Every GPU step has its own limit; a crash / timeout stops the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # step <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  echo "=== $name" | tee -a gpurun_out/final_steps.log
  timeout -k 10 "$t" "$@" > "gpurun_out/final_$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a gpurun_out/final_steps.log
  tail -n 3 "gpurun_out/final_$name.log" | cut -c1-400
  if [ $rc -ne 0 ]; then exit $rc; fi
}
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step tests 700 python -u -m pytest -m gpu -x -q --timeout 150 --timeout-method thread tests
step bench 300 python bench.py
step prof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_final -o run --output-format csv -- python3 bench.py --steps 10 --warmup 5 --no-cpu-baseline
step cnftrain 300 python bench.py --cnf-train --steps 5 --warmup 2
step proftrain 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_cnftrain -o run --output-format csv -- python3 bench.py --cnf-train --steps 3 --warmup 1 --no-cpu-baseline
step nsa16 300 python bench.py --flow nsa16 --batch 1048576
step maf 300 python bench.py --flow maf
exit 0
