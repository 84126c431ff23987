#!/bin/bash
# Round 6, GPU call 2: the spline-VJP tail fix — new tail / multi-step tests, the NaN diagnostic, the train bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
T=${TAG:-r06_g2}
scripts/gpu_steps.sh $T \
  "tests|600|python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_train.py -k 'tail or steps_finite or fused_train'" \
  "diag|300|python -u scripts/diag_train_nan.py --tag $T --steps 40 --trials 4" \
  "train|300|python bench.py --train"
