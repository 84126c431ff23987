#!/bin/bash
# PMC passes for the fused coupling kernel (one counter group per rocprofv3 run, kernel-trace
# domain only — never combined with sys/runtime traces).  Output: gpurun_out/pmc_<TAG>/...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-r01}
OUT=gpurun_out/pmc_$TAG
mkdir -p "$OUT"
ARGS=${ARGS:-"--steps 2 --warmup 1 --no-cpu-baseline"}
timeout -k 10 120 rocprofv3 -L > "$OUT/counters_list.txt" 2>&1
echo "list rc=$?"
i=0
# PMC_GROUPS: counter groups separated by ';' (one rocprofv3 pass each)
DEFAULT_GROUPS="FETCH_SIZE;WRITE_SIZE;SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES GRBM_GUI_ACTIVE;SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_VALU_MFMA_COEXEC_CYCLES SQ_INSTS_VALU_TRANS_F32;SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE TCC_HIT_sum TCC_MISS_sum"
IFS=';' read -r -a GROUP_LIST <<< "${PMC_GROUPS:-$DEFAULT_GROUPS}"
for group in "${GROUP_LIST[@]}"; do
  i=$((i+1))
  echo "=== pass $i: $group"
  # CMD: the profiled program (default: the bench); e.g. CMD="scripts/gemm_bench.py --only fwd2"
  timeout -k 10 300 rocprofv3 --pmc $group -d "$OUT/p$i" -o run --output-format csv -- python3 ${CMD:-bench.py $ARGS} > "$OUT/p$i.log" 2>&1
  rc=$?
  echo "pass $i rc=$rc"
  if [ $rc -ge 124 ]; then echo "stopping (rc=$rc)"; exit $rc; fi
done
exit 0
