#!/bin/bash
# Round 5, GPU call 14: the dW tile kernel's 16-byte loads (gemm_tn128_kernel, vec): the GEMM +
# training suites, the probe, same-box A/Bs against HEAD's library (pre) on the wide-maf step.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
T=${TAG:-r05_g14}
PT="python -u -m pytest -m gpu -x -q --timeout 300 --timeout-method thread"
TR="python bench.py --train --flow maf4 --no-cpu-baseline"
P=$PWD/naz_amd/lib/libnazhip_pre.so
scripts/gpu_steps.sh $T \
  "tests|600|$PT tests/test_gpu_grad.py tests/test_gpu_train.py tests/test_bayes_maf.py" \
  "rg_probe|300|python scripts/rg_wide_probe.py" \
  "maf4_new|300|$TR --steps 5 --warmup 2" \
  "maf4_pre|300|NAZ_LIB=$P $TR --steps 5 --warmup 2" \
  "maf4_new_b|300|$TR --steps 5 --warmup 2" \
  "maf4_pre_b|300|NAZ_LIB=$P $TR --steps 5 --warmup 2" \
  "nb_new|300|$TR --batch 10752 --steps 10 --warmup 3" \
  "nb_pre|300|NAZ_LIB=$P $TR --batch 10752 --steps 10 --warmup 3" \
  "nb_new_b|300|$TR --batch 10752 --steps 10 --warmup 3" \
  "nb_pre_b|300|NAZ_LIB=$P $TR --batch 10752 --steps 10 --warmup 3"
