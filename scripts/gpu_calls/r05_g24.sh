#!/bin/bash
# Round 5, GPU call 24: the config-3 NLL step with the next micro-batch's forward on a second stream
# beside the current backward (NAZ_TRAIN_FWD_STREAM): the training suite, same-box A/Bs twice.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
T=${TAG:-r05_g24}
PT="python -u -m pytest -m gpu -x -q --timeout 300 --timeout-method thread"
TN="python bench.py --train --no-cpu-baseline"
scripts/gpu_steps.sh $T \
  "tests|600|$PT tests/test_gpu_train.py" \
  "train_two|300|$TN" \
  "train_one|300|NAZ_TRAIN_FWD_STREAM=0 $TN" \
  "train_two_b|300|$TN" \
  "train_one_b|300|NAZ_TRAIN_FWD_STREAM=0 $TN"
