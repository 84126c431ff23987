#!/bin/bash
# Round 6, GPU call 3: PMC traffic of the secondary lines (config2, nsa16, nsa, maf), a fresh whole-step
# PMC and kernel trace of the shipped config-3 NLL step, and the side-stream / micro-batch A/Bs on the
# fixed (finite) step.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
T=${TAG:-r06_g3}
O=gpurun_out/$T
P="--steps 2 --warmup 1 --no-cpu-baseline"
steps=()
for fl in config2 nsa16 nsa maf; do
  steps+=("pmcf_$fl|120|rocprofv3 --pmc FETCH_SIZE -d $O/pmc_$fl/p1 -o run --output-format csv -- python3 bench.py --flow $fl $P")
  steps+=("pmcw_$fl|120|rocprofv3 --pmc WRITE_SIZE -d $O/pmc_$fl/p2 -o run --output-format csv -- python3 bench.py --flow $fl $P")
done
TP="--train --steps 1 --warmup 1 --no-cpu-baseline --batch 4194304"
steps+=("pmcf_train|200|rocprofv3 --pmc FETCH_SIZE -d $O/pmc_train/p1 -o run --output-format csv -- python3 bench.py $TP")
steps+=("pmcw_train|200|rocprofv3 --pmc WRITE_SIZE -d $O/pmc_train/p2 -o run --output-format csv -- python3 bench.py $TP")
steps+=("prof_train|200|rocprofv3 --kernel-trace --stats -d $O/prof_train -o run --output-format csv -- python3 bench.py --train --steps 3 --warmup 1 --no-cpu-baseline")
steps+=("mb22_side|200|python bench.py --train --no-cpu-baseline")
steps+=("mb22_one|200|NAZ_TRAIN_DW_STREAM=0 python bench.py --train --no-cpu-baseline")
steps+=("mb20_side|200|python bench.py --train --no-cpu-baseline --micro-batch 1048576")
steps+=("mb20_one|200|NAZ_TRAIN_DW_STREAM=0 python bench.py --train --no-cpu-baseline --micro-batch 1048576")
steps+=("mb23_side|200|python bench.py --train --no-cpu-baseline --micro-batch 8388608")
steps+=("mb22_side_b|200|python bench.py --train --no-cpu-baseline")
steps+=("mb22_one_b|200|NAZ_TRAIN_DW_STREAM=0 python bench.py --train --no-cpu-baseline")
scripts/gpu_steps.sh $T "${steps[@]}"
