#!/bin/bash
# Round 6, GPU call 8: the whole GPU suite on the current tree, then the maf4 minibatch line with r05's
# exact arguments (A/B vs profiles/r05_final4_maf4_nb.json).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
T=${TAG:-r06_g8}
scripts/gpu_steps.sh $T \
  "suite|1100|python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider" \
  "maf4nb|300|python bench.py --train --flow maf4 --no-cpu-baseline --batch 10752 --steps 10 --warmup 3" \
  "maf4nb_g|300|python bench.py --train --flow maf4 --no-cpu-baseline --batch 10752 --steps 10 --warmup 3 --graph"
