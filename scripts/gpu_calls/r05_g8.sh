#!/bin/bash
# Round 5, GPU call 8: nsa16 log_prob A/B of the lane exchanges (HEAD~ library: natural-order row
# values + ds_bpermute; this tree: per-quarter x slices + ds_bpermute; perm: + v_permlane swaps),
# stages spanning passes (span8 / span12: 32 / 48 KB caps), the AR suites on this tree, and the wide maf GEMM shapes alone (rowgemm fill, dW split-K).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
T=${TAG:-r05_g8}
NS="python bench.py --flow nsa16 --no-cpu-baseline --steps 30"
L=$PWD/naz_amd/lib
scripts/gpu_steps.sh $T \
  "ar_tests|600|python -u -m pytest tests/test_gpu_ar_fused.py tests/test_gpu_grad.py -m gpu -x -q --timeout 300 --timeout-method thread" \
  "nsa16_base|200|NAZ_LIB=$L/libnazhip_base.so $NS" \
  "nsa16_x8|200|$NS" \
  "nsa16_perm|200|NAZ_LIB=$L/libnazhip_perm.so $NS" \
  "nsa16_base_b|200|NAZ_LIB=$L/libnazhip_base.so $NS" \
  "nsa16_x8_b|200|$NS" \
  "nsa16_perm_b|200|NAZ_LIB=$L/libnazhip_perm.so $NS" \
  "nsa16_span8|200|NAZ_LIB=$L/libnazhip_span8.so $NS" \
  "nsa16_span12|200|NAZ_LIB=$L/libnazhip_span12.so $NS" \
  "nsa16_span8_b|200|NAZ_LIB=$L/libnazhip_span8.so $NS" \
  "nsa16_span12_b|200|NAZ_LIB=$L/libnazhip_span12.so $NS" \
  "ar_span8_tests|600|NAZ_LIB=$L/libnazhip_span8.so python -u -m pytest tests/test_gpu_ar_fused.py -m gpu -x -q --timeout 300 --timeout-method thread" \
  "nsa4_base|200|NAZ_LIB=$L/libnazhip_base.so python bench.py --flow nsa --no-cpu-baseline --steps 30" \
  "nsa4_x8|200|python bench.py --flow nsa --no-cpu-baseline --steps 30" \
  "maf_base|200|NAZ_LIB=$L/libnazhip_base.so python bench.py --flow maf --no-cpu-baseline --steps 30" \
  "maf_x8|200|python bench.py --flow maf --no-cpu-baseline --steps 30" \
  "rg_probe|300|python scripts/rg_wide_probe.py"
