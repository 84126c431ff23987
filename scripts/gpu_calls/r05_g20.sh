#!/bin/bash
# Round 5, GPU call 20: the wide-maf chain steps' per-degree-block products on parallel streams:
# the training suite (on / off equality, oracle parity, the graphed step), same-box A/Bs of the step at
# 2^16 and 10,752 rows (eager and graphed).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
T=${TAG:-r05_g20}
PT="python -u -m pytest -m gpu -x -q --timeout 300 --timeout-method thread"
TR="python bench.py --train --flow maf4 --no-cpu-baseline"
scripts/gpu_steps.sh $T \
  "tests|600|$PT tests/test_gpu_train.py" \
  "maf4_blk|300|$TR --steps 5 --warmup 2" \
  "maf4_noblk|300|NAZ_MAF_WIDE_BLOCK_STREAMS=0 $TR --steps 5 --warmup 2" \
  "maf4_blk_b|300|$TR --steps 5 --warmup 2" \
  "maf4_noblk_b|300|NAZ_MAF_WIDE_BLOCK_STREAMS=0 $TR --steps 5 --warmup 2" \
  "nb_blk|300|$TR --batch 10752 --steps 10 --warmup 3" \
  "nb_noblk|300|NAZ_MAF_WIDE_BLOCK_STREAMS=0 $TR --batch 10752 --steps 10 --warmup 3" \
  "nb_blk_b|300|$TR --batch 10752 --steps 10 --warmup 3" \
  "nb_noblk_b|300|NAZ_MAF_WIDE_BLOCK_STREAMS=0 $TR --batch 10752 --steps 10 --warmup 3" \
  "nb_blk_graph|300|$TR --batch 10752 --steps 10 --warmup 3 --graph"
