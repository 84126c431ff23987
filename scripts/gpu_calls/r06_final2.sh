#!/bin/bash
# Round 6, closing GPU call: smoke and the whole GPU suite on the final tree (after the empty-slice and
# embedded-context tests), the headline line.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
T=${TAG:-r06_final2}
scripts/gpu_steps.sh $T \
  "smoke|300|python -c 'import __graft_entry__ as g; g.smoke()'" \
  "tests|900|python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider" \
  "bench|300|python bench.py"
