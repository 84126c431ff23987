#!/bin/bash
# Round 6, GPU call 9: what the backward kernel's dW operand stores cost — kernel traces of the config-3
# NLL step with the shipped library and with NAZ_ABL_BWD_NOSTORE (timing only, wrong gradients).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
T=${TAG:-r06_g9}
O=gpurun_out/$T
A="--train --steps 1 --warmup 0 --no-cpu-baseline"
scripts/gpu_steps.sh $T \
  "prof_main|200|rocprofv3 --kernel-trace --stats -d $O/prof_main -o run --output-format csv -- python3 bench.py $A" \
  "prof_nostore|200|NAZ_LIB=$PWD/naz_amd/lib/libnazhip_nostore.so rocprofv3 --kernel-trace --stats -d $O/prof_nostore -o run --output-format csv -- python3 bench.py $A"
