#!/bin/bash
# round 3: the full GPU suite and smoke, as the driver runs them
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/full_smoke.log 2>&1 || { echo "smoke rc=$?"; tail -20 gpurun_out/full_smoke.log; exit 1; }
tail -1 gpurun_out/full_smoke.log
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/full_tests.log 2>&1
rc=$?
tail -5 gpurun_out/full_tests.log
exit $rc
