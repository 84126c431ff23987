#!/bin/bash
# Round 6, GPU call 6: the B-resident f16x3 batch-row GEMM — correctness (rowgemm tests) and a probe
# against the FP32 rowgemm / h3 at the CNF and wide-maf shapes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
T=${TAG:-r06_g6}
scripts/gpu_steps.sh $T \
  "rg_tests|300|python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_grad.py -k 'rowgemm_panel_split'" \
  "probe|300|python -u scripts/bres_probe.py"
