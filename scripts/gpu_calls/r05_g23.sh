#!/bin/bash
# Round 5, GPU call 23: CNF training with the next RK4 step's forward recompute prefetched on its own
# stream (NAZ_CNF_PREFETCH): the CNF suites, same-box A/Bs of the step twice.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
T=${TAG:-r05_g23}
PT="python -u -m pytest -m gpu -x -q --timeout 300 --timeout-method thread"
CT="python bench.py --cnf-train --no-cpu-baseline --steps 5 --warmup 2"
scripts/gpu_steps.sh $T \
  "tests|600|$PT tests/test_gpu_cnf_grad.py tests/test_gpu_cnf_walk.py" \
  "cnf_pre|300|$CT" \
  "cnf_nopre|300|NAZ_CNF_PREFETCH=0 $CT" \
  "cnf_pre_b|300|$CT" \
  "cnf_nopre_b|300|NAZ_CNF_PREFETCH=0 $CT"
