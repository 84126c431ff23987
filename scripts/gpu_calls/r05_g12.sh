#!/bin/bash
# Round 5, GPU call 12: the f16x3 batch-row GEMM (naz_tuning "rowgemm_h3"): GEMM tests on every
# arithmetic, the wide-maf / CNF gradient suites with it on, the GEMM probe with it on, same-box A/Bs
# of the wide-maf NLL step (2^16 rows and naz's 10,752-row minibatch) and the CNF training step.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
T=${TAG:-r05_g12}
PT="python -u -m pytest -m gpu -x -q --timeout 300 --timeout-method thread"
TR="python bench.py --train --flow maf4 --no-cpu-baseline"
CT="python bench.py --cnf-train --no-cpu-baseline --steps 5 --warmup 2"
scripts/gpu_steps.sh $T \
  "grad_tests|600|$PT tests/test_gpu_grad.py" \
  "h3_train_tests|600|NAZ_RG_H3=1 $PT tests/test_gpu_train.py -k 'maf or wide' tests/test_gpu_cnf_grad.py tests/test_gpu_cnf_walk.py" \
  "rg_probe_h3|300|NAZ_RG_H3=1 python scripts/rg_wide_probe.py" \
  "maf4_fp32|300|$TR --steps 5 --warmup 2" \
  "maf4_h3|300|NAZ_RG_H3=1 $TR --steps 5 --warmup 2" \
  "maf4_fp32_b|300|$TR --steps 5 --warmup 2" \
  "maf4_h3_b|300|NAZ_RG_H3=1 $TR --steps 5 --warmup 2" \
  "nb_fp32|300|$TR --batch 10752 --steps 10 --warmup 3" \
  "nb_h3|300|NAZ_RG_H3=1 $TR --batch 10752 --steps 10 --warmup 3" \
  "cnf_fp32|300|$CT" \
  "cnf_h3|300|NAZ_RG_H3=1 $CT"
