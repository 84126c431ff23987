#!/bin/bash
# A/B the bench over library variants: VARIANTS="base A B" -> naz_amd/lib/libnazhip[_X].so
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for rep in 1 2; do
for v in ${VARIANTS:-base}; do
  lib=naz_amd/lib/libnazhip.so; [ "$v" != base ] && lib=naz_amd/lib/libnazhip_$v.so
  NAZ_LIB=$PWD/$lib timeout -k 10 120 python bench.py --no-cpu-baseline --steps 30 ${BENCH_ARGS:-} > gpurun_out/ab_$v.log 2>&1
  rc=$?; if [ $rc -ge 124 ]; then echo "stop $v rc=$rc"; exit $rc; fi
  python3 -c "import json,sys; d=json.loads([l for l in open('gpurun_out/ab_$v.log') if l.startswith('{')][0]); print('$v', round(d['roofline']['avg_kernel_ms'],4), round(d['value']/1e6,1))"
done; done
