#!/bin/bash
# Round 6, GPU call 13: non-temporal stores for the backward's dW operands nothing re-reads
# (NAZ_BWD_NT_STORES variant library) vs the shipped library, interleaved, config-3 NLL step.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
T=${TAG:-r06_g13}
NT="NAZ_LIB=$PWD/naz_amd/lib/libnazhip_ntst.so"
scripts/gpu_steps.sh $T \
  "main1|200|python bench.py --train --no-cpu-baseline" \
  "nt1|200|$NT python bench.py --train --no-cpu-baseline" \
  "main2|200|python bench.py --train --no-cpu-baseline" \
  "nt2|200|$NT python bench.py --train --no-cpu-baseline"
