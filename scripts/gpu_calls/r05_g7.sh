#!/bin/bash
# Round 5, GPU call 7: the whole GPU suite on the AR inverse's per-quarter x slices + permlane
# exchanges and the batch-row GEMM's small-batch grid fill; same-box A/Bs: nsa16 log_prob (HEAD
# library / this tree / two tiles per wave), the wide-maf NLL step at naz's 10,752-row minibatch and
# at 2^16 rows over the fill setting; a kernel trace of the 10,752-row step.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
T=${TAG:-r05_g7}
TR="python bench.py --train --flow maf4 --no-cpu-baseline"
NS="python bench.py --flow nsa16 --no-cpu-baseline --steps 30"
L=$PWD/naz_amd/lib
scripts/gpu_steps.sh $T \
  "smoke|300|python -c 'import __graft_entry__ as g; g.smoke()'" \
  "tests|900|python -u -m pytest ${TESTS:-tests} -m gpu -x -q --timeout 300 --timeout-method thread" \
  "nsa16_base|200|NAZ_LIB=$L/libnazhip_base.so $NS" \
  "nsa16_new|200|$NS" \
  "nsa16_nt2|200|NAZ_LIB=$L/libnazhip_nt2.so $NS" \
  "nsa16_base_b|200|NAZ_LIB=$L/libnazhip_base.so $NS" \
  "nsa16_new_b|200|$NS" \
  "nb_fill0|300|NAZ_RG_FILL=0 $TR --batch 10752 --steps 10 --warmup 3" \
  "nb_fill2|300|$TR --batch 10752 --steps 10 --warmup 3" \
  "nb_fill4|300|NAZ_RG_FILL=4 $TR --batch 10752 --steps 10 --warmup 3" \
  "nb_fill0_b|300|NAZ_RG_FILL=0 $TR --batch 10752 --steps 10 --warmup 3" \
  "nb_fill2_b|300|$TR --batch 10752 --steps 10 --warmup 3" \
  "maf4_fill0|300|NAZ_RG_FILL=0 $TR --steps 5 --warmup 2" \
  "maf4_fill2|300|$TR --steps 5 --warmup 2" \
  "nb_trace|300|rocprofv3 --kernel-trace --stats -d gpurun_out/$T/nb_prof -o nb -- python bench.py --train --flow maf4 --no-cpu-baseline --batch 10752 --steps 10 --warmup 3"
