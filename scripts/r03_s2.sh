#!/bin/bash
# round 3, session 2: parity of the new split / buffer-DMA build, same-box A/B of the variants,
# steady-state kernel trace of the shipped headline kernel, its PMC passes, the exact-FP32 line.
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
step parity 500 python -u -m pytest -m gpu -x -q --timeout 150 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_flow_abi.py tests/test_gpu_cnf.py
VARIANTS="base glds nowait nocopy" step ab 600 bash scripts/ab.sh
step prof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_s2 -o run --output-format csv -- python3 bench.py --steps 30 --warmup 10 --no-cpu-baseline
TAG=r03_headline ARGS="--steps 3 --warmup 2 --no-cpu-baseline" step pmc 600 bash scripts/pmc.sh
step f32 300 python bench.py --mfma f32 --steps 10 --warmup 3
step dp5g 300 python bench.py --cnf --cnf-solver dopri5 --steps 5 --warmup 2
step dp5grp 300 python bench.py --cnf --cnf-solver dopri5 --cnf-control group --steps 5 --warmup 2 --no-cpu-baseline
exit 0
