#!/bin/bash
# round 3, session 24: bf16x6 dW with the grid-interleaved chunk order — dW / gradient tests, the dW
# probe, then the training step and the NUTS gradient vs contiguous row blocks (NAZ_WGRAD_INTERLEAVE=0)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/s24_$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/s24_$name.log | head -1)" | tee -a gpurun_out/s24_steps.log
  tail -n 2 "gpurun_out/s24_$name.log" | cut -c1-300
  if [ $rc -ne 0 ]; then exit $rc; fi
}
step tests 900 python -u -m pytest tests/test_gpu_grad.py tests/test_gpu_train.py tests/test_bayes_maf.py -x -q -m gpu --timeout 300 --timeout-method thread
WG_TORCH=0 step probe_il 200 python scripts/wgrad_probe.py
NAZ_WGRAD_INTERLEAVE=0 WG_TORCH=0 step probe_blk 200 python scripts/wgrad_probe.py
for rep in 1 2; do
  step train_il_$rep 300 python bench.py --train --steps 3 --warmup 1 --no-cpu-baseline
  NAZ_WGRAD_INTERLEAVE=0 step train_blk_$rep 300 python bench.py --train --steps 3 --warmup 1 --no-cpu-baseline
done
step grad_il 300 python bench.py --bayes grad --no-cpu-baseline
NAZ_WGRAD_INTERLEAVE=0 step grad_blk 300 python bench.py --bayes grad --no-cpu-baseline
exit 0
