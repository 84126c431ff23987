#!/bin/bash
# Round 5, GPU call 2: the whole GPU suite on the ABI-3 image registry / workspace / panel-split tree,
# then the wide-maf NLL step with the rowgemm panel split on (default) and off (same-box A/B).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
T=${TAG:-r05_g2}
scripts/gpu_steps.sh $T \
  "smoke|300|python -c 'import __graft_entry__ as g; g.smoke()'" \
  "tests|900|python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
  "bench|300|python bench.py" \
  "train_maf4_split|300|python bench.py --train --flow maf4 --steps 5 --warmup 2 --no-cpu-baseline" \
  "train_maf4_nosplit|300|NAZ_RG_SPLIT=0 python bench.py --train --flow maf4 --steps 5 --warmup 2 --no-cpu-baseline" \
  "train_maf4_split_b|300|python bench.py --train --flow maf4 --steps 5 --warmup 2 --no-cpu-baseline" \
  "train_maf4_nosplit_b|300|NAZ_RG_SPLIT=0 python bench.py --train --flow maf4 --steps 5 --warmup 2 --no-cpu-baseline"
