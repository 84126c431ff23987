#!/bin/bash
# round 3 final measurement set (session 3): smoke, the GPU suite, the headline + its kernel trace,
# the training step, the NUTS gradient, the train step's kernel trace and the AR sampler lines
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/f3_$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/f3_$name.log | head -1)" | tee -a gpurun_out/f3_steps.log
  tail -n 2 "gpurun_out/f3_$name.log" | cut -c1-200
  if [ $rc -ne 0 ]; then exit $rc; fi
}
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step tests 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread
step bench 300 python bench.py
step bench_prof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_f3 -o run --output-format csv -- python3 bench.py --steps 30 --warmup 10 --no-cpu-baseline
step train 400 python bench.py --train --steps 3 --warmup 1
step train_prof 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_f3t -o run --output-format csv -- python3 bench.py --train --steps 2 --warmup 1 --no-cpu-baseline
step bayes_grad 300 python bench.py --bayes grad --steps 10 --warmup 3
step nsa16_sample 300 python bench.py --flow nsa16 --sample
step maf_sample 300 python bench.py --flow maf --sample
step maf4_sample 300 python bench.py --flow maf4 --sample --no-cpu-baseline
exit 0
