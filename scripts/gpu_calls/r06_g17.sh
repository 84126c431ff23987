#!/bin/bash
# Round 6, GPU call 17: bench.py's time-floored warm-up (>= --warmup steps and >= 50 ms) at the
# per-rank slices of the strong-scaling runs (2^17 rows = N 8, 2^18 = N 4) and the full batch.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
T=${TAG:-r06_g17}
scripts/gpu_steps.sh $T \
  "lp_n1|200|python bench.py --no-cpu-baseline" \
  "lp_b18|200|python bench.py --no-cpu-baseline --batch 262144" \
  "lp_b17|200|python bench.py --no-cpu-baseline --batch 131072" \
  "lp_b17_b|200|python bench.py --no-cpu-baseline --batch 131072" \
  "c2_n1|200|python bench.py --flow config2 --no-cpu-baseline" \
  "c2_b15|200|python bench.py --flow config2 --no-cpu-baseline --batch 32768"
