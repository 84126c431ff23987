#!/bin/bash
# Round 6, GPU call 12: the backward kernel's compute at one wave per SIMD (what a fused-dW kernel, which
# needs the register file of a whole SIMD for its accumulators, would run at): kernel traces of the
# config-3 NLL step with the shipped library, NAZ_ABL_BWD_NOSTORE, and NOSTORE + NAZ_ABL_BWD_ONEWG.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
T=${TAG:-r06_g12}
O=gpurun_out/$T
A="--train --steps 1 --warmup 0 --no-cpu-baseline"
R="rocprofv3 --kernel-trace --stats -o run --output-format csv"
scripts/gpu_steps.sh $T \
  "prof_main|200|$R -d $O/prof_main -- python3 bench.py $A" \
  "prof_nostore|200|NAZ_LIB=$PWD/naz_amd/lib/libnazhip_nostore.so $R -d $O/prof_nostore -- python3 bench.py $A" \
  "prof_onewg|200|NAZ_LIB=$PWD/naz_amd/lib/libnazhip_onewg.so $R -d $O/prof_onewg -- python3 bench.py $A"
