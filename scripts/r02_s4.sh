#!/bin/bash
# resident-weight rowgemm: A/B microbench, GPU suite, CNF-train line
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
echo "== resident" && timeout -k 10 120 python scripts/rg_res_bench.py || exit $?
echo "== staged" && NAZ_RG_RESIDENT=0 timeout -k 10 120 python scripts/rg_res_bench.py || exit $?
timeout -k 10 700 python -u -m pytest -m gpu -x -q --timeout 150 --timeout-method thread tests > gpurun_out/s4_tests.log 2>&1
rc=$?
tail -15 gpurun_out/s4_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --cnf-train --steps 5 --warmup 2 > gpurun_out/bench_cnf_train.log 2>&1 || exit $?
grep '^{' gpurun_out/bench_cnf_train.log | cut -c1-300
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_cnf_train2 -o run --output-format csv -- python3 bench.py --cnf-train --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/prof_cnf_train2.log 2>&1 || exit $?
exit 0
