#!/bin/bash
# Round 5, GPU call 13: the batch-row GEMM's branch-free B / mask loads (exact buffer ranges, mask
# applied at the LDS store): GEMM + training suites, the probe, same-box A/Bs against the previous
# commit's library (c05) on the wide-maf step (2^16, 10,752 rows) and the CNF training step.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
T=${TAG:-r05_g13}
PT="python -u -m pytest -m gpu -x -q --timeout 300 --timeout-method thread"
TR="python bench.py --train --flow maf4 --no-cpu-baseline"
CT="python bench.py --cnf-train --no-cpu-baseline --steps 5 --warmup 2"
C=$PWD/naz_amd/lib/libnazhip_c05.so
scripts/gpu_steps.sh $T \
  "tests|600|$PT tests/test_gpu_grad.py tests/test_gpu_train.py tests/test_gpu_cnf_grad.py tests/test_gpu_cnf_walk.py" \
  "rg_probe|300|python scripts/rg_wide_probe.py" \
  "maf4_new|300|$TR --steps 5 --warmup 2" \
  "maf4_c05|300|NAZ_LIB=$C $TR --steps 5 --warmup 2" \
  "maf4_new_b|300|$TR --steps 5 --warmup 2" \
  "maf4_c05_b|300|NAZ_LIB=$C $TR --steps 5 --warmup 2" \
  "nb_new|300|$TR --batch 10752 --steps 10 --warmup 3" \
  "nb_c05|300|NAZ_LIB=$C $TR --batch 10752 --steps 10 --warmup 3" \
  "cnf_new|300|$CT" \
  "cnf_c05|300|NAZ_LIB=$C $CT" \
  "cnf_new_b|300|$CT" \
  "cnf_c05_b|300|NAZ_LIB=$C $CT"
