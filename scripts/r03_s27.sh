#!/bin/bash
# round 3, session 27: compiler-flag A/B of the shipped sources (same box): default vs the max-ILP
# machine scheduler vs flushed denormals — headline and training step
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
L=$PWD/naz_amd/lib
run() {
  local name=$1 lib=$2; shift 2
  NAZ_LIB=$lib timeout -k 10 300 python bench.py "$@" --no-cpu-baseline > gpurun_out/s27_$name.log 2>&1 || { echo "$name failed"; tail -3 gpurun_out/s27_$name.log; exit 1; }
  echo "=== $name $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/s27_$name.log | head -1)"
}
for rep in 1 2; do
  run head_def_$rep $L/libnazhip.so --steps 30 --warmup 10
  run head_ilp_$rep $L/libnazhip_ilp.so --steps 30 --warmup 10
  run head_ftz_$rep $L/libnazhip_ftz.so --steps 30 --warmup 10
done
run train_def $L/libnazhip.so --train --steps 3 --warmup 1
run train_ilp $L/libnazhip_ilp.so --train --steps 3 --warmup 1
run train_ftz $L/libnazhip_ftz.so --train --steps 3 --warmup 1
exit 0
