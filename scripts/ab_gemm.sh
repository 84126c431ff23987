#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for v in ${VARIANTS:-base}; do
  lib=naz_amd/lib/libnazhip.so; [ "$v" != base ] && lib=naz_amd/lib/libnazhip_$v.so
  echo "== $v"; NAZ_LIB=$PWD/$lib timeout -k 10 120 python scripts/gemm_bench.py || exit $?
done
