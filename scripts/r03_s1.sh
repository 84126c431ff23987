#!/bin/bash
# round 3, session 1: the ring-barrier fix — smoke, the whole GPU suite, then the headline
# before (r02 library) / after (ring_barrier) A/B on the same box.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # step <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  echo "=== $name" | tee -a gpurun_out/s1_steps.log
  timeout -k 10 "$t" "$@" > "gpurun_out/s1_$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a gpurun_out/s1_steps.log
  tail -n 3 "gpurun_out/s1_$name.log" | cut -c1-400
  if [ $rc -ne 0 ]; then exit $rc; fi
}
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step tests 700 python -u -m pytest -m gpu -q --timeout 150 --timeout-method thread tests
VARIANTS="base r02old" step ab 400 bash scripts/ab.sh
exit 0
