#!/bin/bash
# training bench + kernel trace of the fused NLL step
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 240 python bench.py --train --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r02_train2.json 2> gpurun_out/r02_train2.err || { tail -20 gpurun_out/r02_train2.err; exit 1; }
cat gpurun_out/r02_train2.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_train -o run --output-format csv -- python3 bench.py --train --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/prof_train.log 2>&1 || { tail -20 gpurun_out/prof_train.log; exit 1; }
find gpurun_out/prof_train -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} gpurun_out/train_kernel_stats.csv
python3 scripts/kernel_table.py gpurun_out/train_kernel_stats.csv 2>/dev/null | head -20 || head -12 gpurun_out/train_kernel_stats.csv
