#!/bin/bash
# Round 5, GPU call 9: the batch-row GEMM's balanced <= 4-block panels and fill 4 (default) — the whole
# GPU suite, the bench, same-box A/Bs of the wide-maf NLL step (2^16 rows, naz's 10,752-row minibatch)
# and the CNF training step against the round's first library (half-width split, no fill), the GEMM
# probe, and kernel traces of both wide-maf steps.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
T=${TAG:-r05_g9}
TR="python bench.py --train --flow maf4 --no-cpu-baseline"
CT="python bench.py --cnf-train --no-cpu-baseline --steps 5 --warmup 2"
B=$PWD/naz_amd/lib/libnazhip_base.so
scripts/gpu_steps.sh $T \
  "smoke|300|python -c 'import __graft_entry__ as g; g.smoke()'" \
  "tests|900|python -u -m pytest ${TESTS:-tests} -m gpu -x -q --timeout 300 --timeout-method thread" \
  "bench|300|python bench.py" \
  "maf4_new|300|$TR --steps 5 --warmup 2" \
  "maf4_base|300|NAZ_LIB=$B $TR --steps 5 --warmup 2" \
  "maf4_new_b|300|$TR --steps 5 --warmup 2" \
  "maf4_base_b|300|NAZ_LIB=$B $TR --steps 5 --warmup 2" \
  "nb_new|300|$TR --batch 10752 --steps 10 --warmup 3" \
  "nb_base|300|NAZ_LIB=$B $TR --batch 10752 --steps 10 --warmup 3" \
  "nb_graph|300|$TR --batch 10752 --steps 10 --warmup 3 --graph" \
  "cnf_new|300|$CT" \
  "cnf_base|300|NAZ_LIB=$B $CT" \
  "rg_probe|300|python scripts/rg_wide_probe.py" \
  "maf4_trace|300|rocprofv3 --kernel-trace --stats -d gpurun_out/$T/maf4_prof -o maf4 -- python bench.py --train --flow maf4 --no-cpu-baseline --steps 5 --warmup 2" \
  "nb_trace|300|rocprofv3 --kernel-trace --stats -d gpurun_out/$T/nb_prof -o nb -- python bench.py --train --flow maf4 --no-cpu-baseline --batch 10752 --steps 10 --warmup 3"
