#!/bin/bash
# A/B of the fused training step over library variants + gradient tests of the variant
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in ${VARIANTS:-base}; do
  lib=naz_amd/lib/libnazhip.so; [ "$v" != base ] && lib=naz_amd/lib/libnazhip_$v.so
  NAZ_LIB=$PWD/$lib timeout -k 10 200 python bench.py --train --steps 3 --warmup 1 --no-cpu-baseline --batch 2097152 > gpurun_out/abt_$v.log 2>&1
  rc=$?; if [ $rc -ge 124 ]; then echo "stop $v rc=$rc"; exit $rc; fi
  python3 -c "import json; d=json.loads([l for l in open('gpurun_out/abt_$v.log') if l.startswith('{')][0]); print('$v', round(d['ms_per_step']/2,2), 'ms per 2^20 rows')"
done
for v in ${TESTVARIANTS:-}; do
  lib=naz_amd/lib/libnazhip_$v.so
  NAZ_LIB=$PWD/$lib timeout -k 10 300 python -u -m pytest -m gpu -q --timeout 120 --timeout-method thread tests/test_gpu_grad.py tests/test_gpu_train.py -k "nll_gradient or config3 or fused_train" > gpurun_out/abtest_$v.log 2>&1
  echo "tests $v rc=$?"; grep -E "passed|failed|q99 rel|median rel|max rel" gpurun_out/abtest_$v.log | cut -c1-400 | tail -12
done
