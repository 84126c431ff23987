#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 200 python scripts/diag_mafgrad.py 1500 > gpurun_out/s11_diag.log 2>&1; rc=$?
cat gpurun_out/s11_diag.log | tail -20
exit $rc
