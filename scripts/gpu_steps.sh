#!/bin/bash
# One gpurun session as a list of steps, each under its own time limit, stopping at the first
# failure (exit status, abort, fault or timeout: nothing more runs on the GPU in this call).
#
#   scripts/gpu_steps.sh TAG 'name|seconds|command' ['name|seconds|command' ...]
#
# Each step's output goes to gpurun_out/TAG/<name>.log; a one-line summary per step (exit code and
# the bench line's ms_per_step, if any) is appended to gpurun_out/TAG/steps.log and printed.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=$1; shift
O=gpurun_out/$TAG
mkdir -p "$O"
for spec in "$@"; do
  name=${spec%%|*}; rest=${spec#*|}; t=${rest%%|*}; cmd=${rest#*|}
  start=$(date +%s)
  timeout -k 10 "$t" bash -c "$cmd" > "$O/$name.log" 2>&1
  rc=$?
  ms=$(grep -o '"ms_per_step": [0-9.]*' "$O/$name.log" | tail -1)
  line="=== $name rc=$rc $(( $(date +%s) - start ))s $ms"
  echo "$line" | tee -a "$O/steps.log"
  tail -n 3 "$O/$name.log" | cut -c1-300
  if [ $rc -ne 0 ]; then echo "stopping after $name"; exit $rc; fi
done
exit 0
