#!/bin/bash
# Round 5, GPU call 26: the config-3 NLL step's micro-batch size (2^20 default, 2^21, 2^22 rows) with the
# side-stream dW overlap, same box.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
T=${TAG:-r05_g26}
TN="python bench.py --train --no-cpu-baseline"
scripts/gpu_steps.sh $T \
  "mb20|300|$TN" \
  "mb21|300|$TN --micro-batch 2097152" \
  "mb22|300|$TN --micro-batch 4194304" \
  "mb20_b|300|$TN" \
  "mb21_b|300|$TN --micro-batch 2097152"
