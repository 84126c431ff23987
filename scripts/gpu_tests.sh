#!/bin/bash
# run a subset (or all) of the GPU tests on the box: scripts/gpu_tests.sh [pytest args...]
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -m gpu -x -q --timeout 120 --timeout-method thread "${@:-tests}" > gpurun_out/gpu_tests.log 2>&1
rc=$?
tail -40 gpurun_out/gpu_tests.log
exit $rc
