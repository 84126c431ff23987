#!/bin/bash
# Round 5, GPU call 15: the batch-row GEMM's k-paired LDS chunk images (two ds_read_b128 per operand
# row per chunk): the GEMM / training / CNF / Bayesian suites, the probe, same-box A/Bs against the
# same tree built with the old [k][row] images (v1) on the wide-maf step and CNF training.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
T=${TAG:-r05_g15}
PT="python -u -m pytest -m gpu -x -q --timeout 300 --timeout-method thread"
TR="python bench.py --train --flow maf4 --no-cpu-baseline"
CT="python bench.py --cnf-train --no-cpu-baseline --steps 5 --warmup 2"
V=$PWD/naz_amd/lib/libnazhip_v1.so
scripts/gpu_steps.sh $T \
  "tests|600|$PT tests/test_gpu_grad.py tests/test_gpu_train.py tests/test_bayes_maf.py tests/test_gpu_cnf_grad.py tests/test_gpu_cnf_walk.py" \
  "rg_probe|300|python scripts/rg_wide_probe.py" \
  "maf4_new|300|$TR --steps 5 --warmup 2" \
  "maf4_v1|300|NAZ_LIB=$V $TR --steps 5 --warmup 2" \
  "maf4_new_b|300|$TR --steps 5 --warmup 2" \
  "maf4_v1_b|300|NAZ_LIB=$V $TR --steps 5 --warmup 2" \
  "nb_new|300|$TR --batch 10752 --steps 10 --warmup 3" \
  "nb_v1|300|NAZ_LIB=$V $TR --batch 10752 --steps 10 --warmup 3" \
  "cnf_new|300|$CT" \
  "cnf_v1|300|NAZ_LIB=$V $CT" \
  "cnf_new_b|300|$CT" \
  "cnf_v1_b|300|NAZ_LIB=$V $CT"
