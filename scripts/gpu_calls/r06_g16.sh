#!/bin/bash
# Round 6, GPU call 16: the per-rank work of the driver's strong-scaling runs on one GPU — log_prob at
# the 2^19 / 2^18 / 2^17-row slices of the 2^20 global batch (N = 2 / 4 / 8) and the NLL step at the
# 2^20-row slice of 2^23 (N = 8), beside the N = 1 lines.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
T=${TAG:-r06_g16}
scripts/gpu_steps.sh $T \
  "lp_n1|200|python bench.py --no-cpu-baseline" \
  "lp_b19|200|python bench.py --no-cpu-baseline --batch 524288" \
  "lp_b18|200|python bench.py --no-cpu-baseline --batch 262144" \
  "lp_b17|200|python bench.py --no-cpu-baseline --batch 131072" \
  "lp_b17_s100|200|python bench.py --no-cpu-baseline --batch 131072 --steps 100 --warmup 20" \
  "train_b20|300|python bench.py --train --no-cpu-baseline --batch 1048576"
