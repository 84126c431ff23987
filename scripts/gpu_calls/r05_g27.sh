#!/bin/bash
# Round 5, GPU call 27: the config-3 NLL step at 2^22- and 2^23-row micro-batches (one or two passes over
# the 2^23-row global batch) against 2^20, same box, twice.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
T=${TAG:-r05_g27}
TN="python bench.py --train --no-cpu-baseline"
scripts/gpu_steps.sh $T \
  "mb22|300|$TN --micro-batch 4194304" \
  "mb23|300|$TN --micro-batch 8388608" \
  "mb20|300|$TN" \
  "mb22_b|300|$TN --micro-batch 4194304" \
  "mb23_b|300|$TN --micro-batch 8388608"
