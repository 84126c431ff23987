#!/bin/bash
# A/B the training-step bench over library variants: VARIANTS="base A" -> libnazhip[_A].so
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in ${VARIANTS:-base}; do
  lib=naz_amd/lib/libnazhip.so; [ "$v" != base ] && lib=naz_amd/lib/libnazhip_$v.so
  NAZ_LIB=$PWD/$lib timeout -k 10 200 python bench.py --train --no-cpu-baseline --steps 4 --warmup 1 > gpurun_out/abt_$v.log 2>&1
  rc=$?; if [ $rc -ge 124 ]; then echo "stop $v rc=$rc"; exit $rc; fi
  python3 -c "import json; d=json.loads([l for l in open('gpurun_out/abt_$v.log') if l.startswith('{')][0]); print('$v', round(d['ms_per_step'],2))"
done
