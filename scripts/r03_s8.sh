#!/bin/bash
# round 3, session 8: backward-kernel load placement A/B (train step), then the full GPU suite
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
  local name=$1 t=$2; shift 2
  echo "=== $name" | tee -a gpurun_out/s8_steps.log
  timeout -k 10 "$t" "$@" > "gpurun_out/s8_$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a gpurun_out/s8_steps.log
  tail -n 3 "gpurun_out/s8_$name.log" | cut -c1-300
  if [ $rc -ne 0 ]; then exit $rc; fi
}
for rep in 1 2; do
  step train_new$rep 300 python bench.py --train --steps 3 --warmup 1 --no-cpu-baseline
  NAZ_LIB=$PWD/naz_amd/lib/libnazhip_late.so step train_late$rep 300 python bench.py --train --steps 3 --warmup 1 --no-cpu-baseline
done
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step tests 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread
exit 0
