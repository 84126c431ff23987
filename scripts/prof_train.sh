#!/bin/bash
# rocprofv3 kernel trace of the training bench; per-kernel/grid summary to stdout.
# Usage: LIBV=<variant|base> TAG=<name> bash scripts/prof_train.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
lib=naz_amd/lib/libnazhip.so; [ "${LIBV:-base}" != base ] && lib=naz_amd/lib/libnazhip_$LIBV.so
NAZ_LIB=$PWD/$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG:-t} -o run --output-format csv -- python3 bench.py --train --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/prof_${TAG:-t}.log 2>&1
rc=$?; echo "prof rc=$rc"; [ $rc -ne 0 ] && exit $rc
python3 scripts/kernel_table.py gpurun_out/prof_${TAG:-t}/run_kernel_trace.csv 4
