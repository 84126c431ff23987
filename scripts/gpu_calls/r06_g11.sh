#!/bin/bash
# Round 6, GPU call 11: a 2-rank rehearsal of the multi-GPU bench paths (gloo, both ranks on the one GPU):
# the self-launch, strong-scaling shards, max-over-ranks timing, the DP training all-reduce.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
T=${TAG:-r06_g11}
scripts/gpu_steps.sh $T \
  "rehearse_lp|300|NAZ_BENCH_BACKEND=gloo python bench.py --gpus 2 --steps 5 --warmup 2 --no-cpu-baseline" \
  "rehearse_train|300|NAZ_BENCH_BACKEND=gloo python bench.py --gpus 2 --train --steps 3 --warmup 1 --no-cpu-baseline" \
  "rehearse_cnf|300|NAZ_BENCH_BACKEND=gloo python bench.py --gpus 2 --cnf --steps 3 --warmup 1 --no-cpu-baseline"
