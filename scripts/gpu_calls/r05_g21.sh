#!/bin/bash
# Round 5, GPU call 21: the CNF VJP's weight / bias reductions on a side stream (NAZ_CNF_DW_STREAM): the
# CNF gradient / walk suites, same-box A/Bs of the CNF training step (config 5) twice.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
T=${TAG:-r05_g21}
PT="python -u -m pytest -m gpu -x -q --timeout 300 --timeout-method thread"
CT="python bench.py --cnf-train --no-cpu-baseline --steps 5 --warmup 2"
scripts/gpu_steps.sh $T \
  "tests|600|$PT tests/test_gpu_cnf_grad.py tests/test_gpu_cnf_walk.py tests/test_gpu_cnf.py" \
  "cnf_side|300|$CT" \
  "cnf_one|300|NAZ_CNF_DW_STREAM=0 $CT" \
  "cnf_side_b|300|$CT" \
  "cnf_one_b|300|NAZ_CNF_DW_STREAM=0 $CT"
