#!/bin/bash
# Round 6, GPU call 4: one dW buffer per backward (no zero fills on the side stream) — gradient tests,
# the train bench with 2 / 3 operand sets and with the side stream off, and a kernel trace.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
T=${TAG:-r06_g4}
O=gpurun_out/$T
scripts/gpu_steps.sh $T \
  "tests|600|python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_train.py -k 'tail or steps_finite or fused_train or micro_batch or dp_two'" \
  "set2|200|python bench.py --train --no-cpu-baseline" \
  "set3|200|NAZ_TRAIN_DW_SETS=3 python bench.py --train --no-cpu-baseline" \
  "one|200|NAZ_TRAIN_DW_STREAM=0 python bench.py --train --no-cpu-baseline" \
  "set2b|200|python bench.py --train --no-cpu-baseline" \
  "set3b|200|NAZ_TRAIN_DW_SETS=3 python bench.py --train --no-cpu-baseline" \
  "mb20|200|python bench.py --train --no-cpu-baseline --micro-batch 1048576" \
  "prof|200|rocprofv3 --kernel-trace --stats -d $O/prof_train -o run --output-format csv -- python3 bench.py --train --steps 3 --warmup 1 --no-cpu-baseline"
