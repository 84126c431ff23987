#!/bin/bash
# Round-end measurement set (one gpurun call): default bench, kernel-trace summary of the same
# command, PMC HBM traffic passes, training and CNF bench lines.  Output under gpurun_out/round/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/round
rm -rf $O/pmc $O/prof $O/prof_cnf $O/prof_train $O/prof_cnf_dopri5 $O/prof_bayes_sample
mkdir -p $O
step() {  # step <name> <timeout> <cmd...>; stop on crash / timeout
  local name=$1 t=$2; shift 2
  echo "=== $name"
  timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "rc=$rc"; tail -n 2 "$O/$name.log" | cut -c1-400
  if [ $rc -ne 0 ]; then echo "stopping after $name"; exit $rc; fi
}
step bench 300 python bench.py
step prof 240 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --steps 20 --warmup 10 --no-cpu-baseline
step pmc_fetch 120 rocprofv3 --pmc FETCH_SIZE -d $O/pmc/p1 -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline
step pmc_write 120 rocprofv3 --pmc WRITE_SIZE -d $O/pmc/p2 -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline
step pmc_sq 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $O/pmc/p3 -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline
step pmc_wait 120 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_VALU_MFMA_COEXEC_CYCLES SQ_INSTS_VALU_TRANS_F32 -d $O/pmc/p4 -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline
step train 300 python bench.py --train --steps 5 --warmup 2
step prof_train 240 rocprofv3 --kernel-trace --stats -d $O/prof_train -o run --output-format csv -- python3 bench.py --train --steps 3 --warmup 1 --no-cpu-baseline
step gemm_bench 120 python scripts/gemm_bench.py
step cnf 300 python bench.py --cnf --steps 10 --warmup 3
step prof_cnf 240 rocprofv3 --kernel-trace --stats -d $O/prof_cnf -o run --output-format csv -- python3 bench.py --cnf --steps 10 --warmup 3
for f in config2 maf nsa maf_grid; do step flow_$f 240 python bench.py --flow $f --steps 10 --warmup 3; done
step cnf_dopri5 300 python bench.py --cnf --cnf-solver dopri5 --steps 10 --warmup 3
step prof_cnf_dopri5 240 rocprofv3 --kernel-trace --stats -d $O/prof_cnf_dopri5 -o run --output-format csv -- python3 bench.py --cnf --cnf-solver dopri5 --steps 10 --warmup 3 --no-cpu-baseline
step bayes_lp 240 python bench.py --bayes lp --steps 10 --warmup 3
step bayes_sample 240 python bench.py --bayes sample --steps 10 --warmup 3
step bayes_grad 240 python bench.py --bayes grad --steps 5 --warmup 2
step prof_bayes_sample 240 rocprofv3 --kernel-trace --stats -d $O/prof_bayes_sample -o run --output-format csv -- python3 bench.py --bayes sample --steps 5 --warmup 2 --no-cpu-baseline
exit 0
