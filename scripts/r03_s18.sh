#!/bin/bash
# round 3, session 17: nsc backward — tanh' epilogues at the next stage's head + preloaded lower-dim
# gradients (default) vs the r02 placement (lowg); gradient tests on the default
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/s18_$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/s18_$name.log | head -1)" | tee -a gpurun_out/s18_steps.log
  tail -n 2 "gpurun_out/s18_$name.log" | cut -c1-200
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
}
L=$PWD/naz_amd/lib
for rep in 1 2; do
  step train_new_$rep 300 python bench.py --train --steps 3 --warmup 1 --no-cpu-baseline
  NAZ_LIB=$L/libnazhip_lowg.so step train_lowg_$rep 300 python bench.py --train --steps 3 --warmup 1 --no-cpu-baseline
done
step tests 600 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_grad.py -x -q -m gpu --timeout 300 --timeout-method thread -k "fused_train or nll_gradient or config3"
exit 0
