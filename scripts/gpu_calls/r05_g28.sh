#!/bin/bash
# Round 5, GPU call 28: the default bench and the config-3 NLL step at its new default micro-batch.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
T=${TAG:-r05_g28}
scripts/gpu_steps.sh $T \
  "smoke|300|python -c 'import __graft_entry__ as g; g.smoke()'" \
  "bench|300|python bench.py" \
  "train|300|python bench.py --train"
