#!/bin/bash
# Round 5, GPU call 25: the batch-row GEMM's grid-fill target under the wide-maf step's three streams
# (NAZ_RG_FILL 2 / 4 (default) / 8) at 2^16 rows and naz's 10,752-row minibatch, and CNF training.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
T=${TAG:-r05_g25}
TR="python bench.py --train --flow maf4 --no-cpu-baseline"
CT="python bench.py --cnf-train --no-cpu-baseline --steps 5 --warmup 2"
scripts/gpu_steps.sh $T \
  "maf4_f4|300|$TR --steps 5 --warmup 2" \
  "maf4_f2|300|NAZ_RG_FILL=2 $TR --steps 5 --warmup 2" \
  "maf4_f8|300|NAZ_RG_FILL=8 $TR --steps 5 --warmup 2" \
  "nb_f4|300|$TR --batch 10752 --steps 10 --warmup 3" \
  "nb_f2|300|NAZ_RG_FILL=2 $TR --batch 10752 --steps 10 --warmup 3" \
  "nb_f8|300|NAZ_RG_FILL=8 $TR --batch 10752 --steps 10 --warmup 3" \
  "cnf_f4|300|$CT" \
  "cnf_f8|300|NAZ_RG_FILL=8 $CT" \
  "maf4_f4_b|300|$TR --steps 5 --warmup 2" \
  "nb_f4_b|300|$TR --batch 10752 --steps 10 --warmup 3"
