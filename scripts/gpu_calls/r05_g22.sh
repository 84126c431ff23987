#!/bin/bash
# Round 5, GPU call 22: the fused maf backward's first-half dW reductions on a side stream
# (NAZ_MAF_DW_STREAM): the Bayesian / maf gradient suites (graph replays included), same-box A/Bs of the
# NUTS potential + gradient (paper shape and the 4-parameter Bayesian MAF), twice.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
T=${TAG:-r05_g22}
PT="python -u -m pytest -m gpu -x -q --timeout 300 --timeout-method thread"
BG="python bench.py --bayes grad --no-cpu-baseline"
scripts/gpu_steps.sh $T \
  "tests|600|$PT tests/test_bayes_maf.py tests/test_gpu_train.py -k 'maf or bayes or grad'" \
  "grad_side|300|$BG" \
  "grad_one|300|NAZ_MAF_DW_STREAM=0 $BG" \
  "grad_side_b|300|$BG" \
  "grad_one_b|300|NAZ_MAF_DW_STREAM=0 $BG" \
  "grad4_side|300|$BG --bayes-shape 4p150" \
  "grad4_one|300|NAZ_MAF_DW_STREAM=0 $BG --bayes-shape 4p150"
