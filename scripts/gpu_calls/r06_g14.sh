#!/bin/bash
# Round 6, GPU call 14: fewer, longer ring stages for the headline kernel (VERDICT r05 Next #3).
# libnazhip_w16s80.so: 16-wave workgroups (256 rows, one per CU) on a 2 x 80 KB ring, so a config-3
# layer is 4 stages (A | B all k-steps | C half 0 | C half 1) instead of 7.  Parity of the variant,
# then same-box interleaved bench lines and a kernel trace of each.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
T=${TAG:-r06_g14}
O=gpurun_out/$T
V="NAZ_LIB=$PWD/naz_amd/lib/libnazhip_w16s80.so"
scripts/gpu_steps.sh $T \
  "parity_v|600|$V python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py" \
  "main1|200|python bench.py --no-cpu-baseline" \
  "v1|200|$V python bench.py --no-cpu-baseline" \
  "main2|200|python bench.py --no-cpu-baseline" \
  "v2|200|$V python bench.py --no-cpu-baseline" \
  "c2_main|200|python bench.py --flow config2 --no-cpu-baseline" \
  "c2_v|200|$V python bench.py --flow config2 --no-cpu-baseline" \
  "kt_v|200|$V rocprofv3 --kernel-trace --stats -d $O/kt_v -o run --output-format csv -- python3 bench.py --no-cpu-baseline"
