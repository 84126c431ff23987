#!/bin/bash
# round 3, session 2: same-box A/B of the ring fix (base vs the racy nowait form), steady-state
# kernel trace of the shipped headline kernel, its PMC passes, and the exact-FP32 line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # step <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  echo "=== $name" | tee -a gpurun_out/s2_steps.log
  timeout -k 10 "$t" "$@" > "gpurun_out/s2_$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a gpurun_out/s2_steps.log
  tail -n 4 "gpurun_out/s2_$name.log" | cut -c1-600
  if [ $rc -ne 0 ]; then exit $rc; fi
}
VARIANTS="base nowait" step ab 400 bash scripts/ab.sh
step prof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_s2 -o run --output-format csv -- python3 bench.py --steps 30 --warmup 10 --no-cpu-baseline
TAG=r03_headline ARGS="--steps 3 --warmup 2 --no-cpu-baseline" step pmc 600 bash scripts/pmc.sh
step f32 300 python bench.py --mfma f32 --steps 10 --warmup 3
exit 0
