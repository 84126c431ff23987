#!/bin/bash
# Round 5, GPU call 11: PMC passes of the wide maf's GEMM kernels at 2^16 rows (K = 512 -> N = 172):
# the batch-row forward (rowgemm_kernel<3>), the chains' dX product, and the dW reduction.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
G1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_INSTS_VMEM GRBM_GUI_ACTIVE"
G2="SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_VALU_TRANS_F32"
G3="FETCH_SIZE"
G4="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE TCC_HIT_sum TCC_MISS_sum"
for op in linear dact dw; do
  O=gpurun_out/r05_g11/$op
  mkdir -p $O
  i=0
  for g in "$G1" "$G2" "$G3" "$G4"; do
    i=$((i+1))
    timeout -k 10 120 rocprofv3 --pmc $g -d $O/p$i -o run --output-format csv -- python3 scripts/rg_pmc_probe.py $op > $O/p$i.log 2>&1
    rc=$?
    echo "$op pass $i rc=$rc"
    if [ $rc -ne 0 ]; then exit $rc; fi
  done
done
exit 0
