#!/bin/bash
# round 3, session 9: smoke, full GPU suite, headline bench and the training step on the restored tree
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
  local name=$1 t=$2; shift 2
  echo "=== $name" | tee -a gpurun_out/s9_steps.log
  timeout -k 10 "$t" "$@" > "gpurun_out/s9_$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a gpurun_out/s9_steps.log
  tail -n 3 "gpurun_out/s9_$name.log" | cut -c1-400
  if [ $rc -ne 0 ]; then exit $rc; fi
}
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step tests 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread
step bench 300 python bench.py
step train 300 python bench.py --train --steps 3 --warmup 1 --no-cpu-baseline
exit 0
