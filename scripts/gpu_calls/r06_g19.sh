#!/bin/bash
# Round 6, GPU call 19 (run on several boxes): the headline line and the sustained clock of its kernel
# (GRBM_GUI_ACTIVE / 8 XCDs over each launch's own duration), to tie the box-to-box spread of the
# headline to the clock each box holds under this load.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
T=${TAG:-r06_g19}
P=gpurun_out/$T
scripts/gpu_steps.sh $T \
  "bench|200|python bench.py --no-cpu-baseline" \
  "pmc_clk|120|rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT -d $P/pmc_clk -o run --output-format csv -- python3 bench.py --steps 10 --warmup 10 --no-cpu-baseline"
