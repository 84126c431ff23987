#!/bin/bash
# Round 6, GPU call 7: dW side stream on / off, interleaved (config-3 NLL step, 2^22-row micro-batches);
# the maf4 and CNF training lines with the per-step loss check; fresh PMC traffic of config2 / nsa16.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
T=${TAG:-r06_g7}
O=gpurun_out/$T
P="--steps 2 --warmup 1 --no-cpu-baseline"
steps=()
for i in 1 2 3; do
  steps+=("side$i|200|NAZ_TRAIN_DW_STREAM=1 python bench.py --train --no-cpu-baseline")
  steps+=("one$i|200|NAZ_TRAIN_DW_STREAM=0 python bench.py --train --no-cpu-baseline")
done
steps+=("maf4|300|python bench.py --train --flow maf4 --no-cpu-baseline")
steps+=("maf4nb|300|python bench.py --train --flow maf4 --batch 10752 --no-cpu-baseline")
steps+=("cnftrain|300|python bench.py --cnf-train --no-cpu-baseline")
for fl in config2 nsa16; do
  steps+=("pmcf_$fl|120|rocprofv3 --pmc FETCH_SIZE -d $O/pmc_$fl/p1 -o run --output-format csv -- python3 bench.py --flow $fl $P")
  steps+=("pmcw_$fl|120|rocprofv3 --pmc WRITE_SIZE -d $O/pmc_$fl/p2 -o run --output-format csv -- python3 bench.py --flow $fl $P")
done
scripts/gpu_steps.sh $T "${steps[@]}"
