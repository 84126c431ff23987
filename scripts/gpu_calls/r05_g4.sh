#!/bin/bash
# Round 5, GPU call 4: the whole GPU suite (ABI-3 image registry / workspace, rowgemm split default on,
# per-layer CNF, graphed NLL step), the bench, the wide-maf NLL step split A/B and at naz's minibatch
# (10,752 rows) eager vs one HIP graph.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
T=${TAG:-r05_g4}
TR="python bench.py --train --flow maf4 --no-cpu-baseline"
scripts/gpu_steps.sh $T \
  "smoke|300|python -c 'import __graft_entry__ as g; g.smoke()'" \
  "tests|900|python -u -m pytest ${TESTS:-tests} -m gpu -x -q --timeout 300 --timeout-method thread" \
  "bench|300|python bench.py" \
  "maf4_split|300|$TR --steps 5 --warmup 2" \
  "maf4_nosplit|300|NAZ_RG_SPLIT=0 $TR --steps 5 --warmup 2" \
  "maf4_split_b|300|$TR --steps 5 --warmup 2" \
  "maf4_nosplit_b|300|NAZ_RG_SPLIT=0 $TR --steps 5 --warmup 2" \
  "maf4_nb_eager|300|$TR --batch 10752 --steps 10 --warmup 3" \
  "maf4_nb_graph|300|$TR --batch 10752 --steps 10 --warmup 3 --graph" \
  "maf4_graph|300|$TR --steps 5 --warmup 2 --graph"
