#!/bin/bash
# Round 5, GPU call 10: the batch-row GEMM's coalesced n-major B loads (the dX products' row-major W):
# GEMM + training suites, the GEMM probe, same-box A/Bs of the wide-maf NLL step against the
# balanced-panel library (p4) and the round's first library (base), kernel traces of both wide-maf
# steps (converted to CSV on the box: the databases exceed the copy-back limit).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
T=${TAG:-r05_g10}
O=gpurun_out/$T
TR="python bench.py --train --flow maf4 --no-cpu-baseline"
L=$PWD/naz_amd/lib
scripts/gpu_steps.sh $T \
  "tests|600|python -u -m pytest tests/test_gpu_grad.py tests/test_gpu_train.py tests/test_gpu_cnf_grad.py -m gpu -x -q --timeout 300 --timeout-method thread" \
  "rg_probe|300|python scripts/rg_wide_probe.py" \
  "maf4_new|300|$TR --steps 5 --warmup 2" \
  "maf4_p4|300|NAZ_LIB=$L/libnazhip_p4.so $TR --steps 5 --warmup 2" \
  "maf4_base|300|NAZ_LIB=$L/libnazhip_base.so $TR --steps 5 --warmup 2" \
  "maf4_new_b|300|$TR --steps 5 --warmup 2" \
  "maf4_p4_b|300|NAZ_LIB=$L/libnazhip_p4.so $TR --steps 5 --warmup 2" \
  "nb_new|300|$TR --batch 10752 --steps 10 --warmup 3" \
  "nb_p4|300|NAZ_LIB=$L/libnazhip_p4.so $TR --batch 10752 --steps 10 --warmup 3" \
  "nb_new_b|300|$TR --batch 10752 --steps 10 --warmup 3" \
  "cnf_new|300|python bench.py --cnf-train --no-cpu-baseline --steps 5 --warmup 2" \
  "maf4_trace|300|rocprofv3 --kernel-trace --stats -d $O/maf4_prof -o maf4 -- python bench.py --train --flow maf4 --no-cpu-baseline --steps 5 --warmup 2" \
  "nb_trace|300|rocprofv3 --kernel-trace --stats -d $O/nb_prof -o nb -- python bench.py --train --flow maf4 --no-cpu-baseline --batch 10752 --steps 10 --warmup 3" \
  "to_csv|120|python scripts/rocpd_stats.py $O/maf4_prof/maf4_results.db $O/maf4_kernel_stats.csv && python scripts/rocpd_stats.py $O/nb_prof/nb_results.db $O/nb_kernel_stats.csv && rm -rf $O/maf4_prof $O/nb_prof"
