#!/bin/bash
# Round 6, GPU call 5: ADVICE fixes (graphed nsc step, uncapturable-flow fallback, workspace cache,
# B == 0 entries), the DP micro-batch cases, the training suite; the flow lines with PMC traffic.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
T=${TAG:-r06_g5}
scripts/gpu_steps.sh $T \
  "train_tests|900|python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_train.py tests/test_gpu_images.py tests/test_gpu_flow_abi.py" \
  "bench|200|python bench.py" \
  "config2|200|python bench.py --flow config2" \
  "nsa16|300|python bench.py --flow nsa16"
