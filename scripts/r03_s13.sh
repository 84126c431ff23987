#!/bin/bash
# round 3, session 13: A/B the training forward at 4 vs 2 waves/SIMD (tw2 = the r02 form) and the
# one-block mixlo split (mix2) on the headline; mix2's parity on the coupling tests
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
  local name=$1 t=$2; shift 2
  echo "=== $name" | tee -a gpurun_out/s13_steps.log
  timeout -k 10 "$t" "$@" > "gpurun_out/s13_$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a gpurun_out/s13_steps.log
  tail -n 6 "gpurun_out/s13_$name.log" | cut -c1-300
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
}
L=$PWD/naz_amd/lib
for rep in 1 2; do
  step train_w4_$rep 300 python bench.py --train --steps 3 --warmup 1 --no-cpu-baseline
  NAZ_LIB=$L/libnazhip_tw2.so step train_w2_$rep 300 python bench.py --train --steps 3 --warmup 1 --no-cpu-baseline
done
step ab_mix2 900 env VARIANTS="base mix2 defA" bash scripts/ab.sh
NAZ_LIB=$L/libnazhip_defA.so step defA_parity 600 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 200 --timeout-method thread -k "flow_log_prob or flow_sample or config3 or ragged or bounds or gemm1 or full_size_exact"
NAZ_LIB=$L/libnazhip_mix2.so step mix2_parity 600 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 200 --timeout-method thread -k "flow_log_prob or flow_sample or config3 or ragged or bounds or gemm1"
step train_tests 600 python -u -m pytest tests/test_gpu_train.py -x -q -m gpu --timeout 300 --timeout-method thread -k "fused_train"
for f in gpurun_out/s13_train_*.log; do echo "$f $(grep -o '"ms_per_step": [0-9.]*' $f)"; done
exit 0
