#!/bin/bash
# Round 5, GPU call 17: the config-3 NLL step with layer l's dW reductions on a side stream overlapping
# layer l + 1's backward (NAZ_TRAIN_DW_STREAM=1): the gradient check against one stream, the training
# suite, and a same-box A/B of the step (2^23 rows), twice.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
T=${TAG:-r05_g17}
PT="python -u -m pytest -m gpu -x -q --timeout 300 --timeout-method thread"
TN="python bench.py --train --no-cpu-baseline"
scripts/gpu_steps.sh $T \
  "tests|600|$PT tests/test_gpu_train.py -k 'side_stream or fused_train or config3'" \
  "train_one|300|$TN" \
  "train_side|300|NAZ_TRAIN_DW_STREAM=1 $TN" \
  "train_one_b|300|$TN" \
  "train_side_b|300|NAZ_TRAIN_DW_STREAM=1 $TN"
