cd "${GRAFT_REPO_ROOT}"
for v in base glds mix32; do
  lib=$PWD/naz_amd/lib/libnazhip.so; [ "$v" != base ] && lib=$PWD/naz_amd/lib/libnazhip_$v.so
  echo "== $v"
  NAZ_LIB=$lib timeout -k 10 120 python -m pytest -m gpu -q --timeout 100 tests/test_gpu_parity.py -k "test_flow_log_prob_vs_golden and nsc" 2>&1 | tail -4
done
