#!/bin/bash
# Round 6, GPU call 10: nsa16 with the context fragments in LDS (no scratch) — AR suite, A/B bench lines,
# PMC; and a 2-rank rehearsal of the multi-GPU bench paths (gloo, both ranks on the one GPU).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
T=${TAG:-r06_g10}
O=gpurun_out/$T
scripts/gpu_steps.sh $T \
  "ar_tests|600|python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_ar_fused.py" \
  "nsa16|200|python bench.py --flow nsa16 --no-cpu-baseline" \
  "nsa16_b|200|python bench.py --flow nsa16 --no-cpu-baseline" \
  "nsa|200|python bench.py --flow nsa --no-cpu-baseline" \
  "pmc_nsa16|200|rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $O/pmc_nsa16/p1 -o run --output-format csv -- python3 bench.py --flow nsa16 --steps 2 --warmup 1 --no-cpu-baseline"
