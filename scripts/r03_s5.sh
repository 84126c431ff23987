#!/bin/bash
# round 3, session 5: the shipped headline kernel — bench line, steady-state kernel trace, PMC
# passes (traffic), nsa16 / maf / train lines on the ring-barrier build
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
  local name=$1 t=$2; shift 2
  echo "=== $name" | tee -a gpurun_out/s5_steps.log
  timeout -k 10 "$t" "$@" > "gpurun_out/s5_$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a gpurun_out/s5_steps.log
  tail -n 3 "gpurun_out/s5_$name.log" | cut -c1-300
  if [ $rc -ne 0 ]; then exit $rc; fi
}
step bench 300 python bench.py
step prof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_s5 -o run --output-format csv -- python3 bench.py --steps 30 --warmup 10 --no-cpu-baseline
TAG=r03_final ARGS="--steps 3 --warmup 2 --no-cpu-baseline" step pmc 600 bash scripts/pmc.sh
step nsa16 300 python bench.py --flow nsa16 --batch 1048576 --no-cpu-baseline
step train 600 python bench.py --train --steps 3 --warmup 1 --no-cpu-baseline
exit 0
