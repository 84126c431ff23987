#!/bin/bash
# Round 5, GPU call 1: the shipped headline kernel's trace + PMC, the configs[1] line, the AR
# inverse (nsa16) PMC.  Output: gpurun_out/r05_g1/ (steps) and gpurun_out/pmc_r05_*/ (PMC passes).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
P=gpurun_out/r05_g1
RP="rocprofv3 --kernel-trace --stats -o run --output-format csv"
scripts/gpu_steps.sh r05_g1 \
  "smoke|300|python -c 'import __graft_entry__ as g; g.smoke()'" \
  "bench|300|python bench.py" \
  "prof_bench|240|$RP -d $P/prof_bench -- python3 bench.py --steps 20 --warmup 10 --no-cpu-baseline" \
  "pmc_bench|600|TAG=r05_headline scripts/pmc.sh" \
  "config2|300|python bench.py --flow config2" \
  "prof_config2|240|$RP -d $P/prof_config2 -- python3 bench.py --flow config2 --steps 20 --warmup 10 --no-cpu-baseline" \
  "pmc_nsa16|600|TAG=r05_nsa16 ARGS='--flow nsa16 --steps 2 --warmup 1 --no-cpu-baseline' scripts/pmc.sh"
