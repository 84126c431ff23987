#!/bin/bash
# HBM traffic passes + kernel-trace summary for the default bench, and a 1-rank torchrun bench
# (exercises the distributed launch path).  Output under gpurun_out/round/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/round
mkdir -p $O
step() {
  local name=$1 t=$2; shift 2
  echo "=== $name"
  timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "rc=$rc"; tail -n 1 "$O/$name.log" | cut -c1-300
  if [ $rc -ne 0 ]; then echo "stopping after $name"; exit $rc; fi
}
rm -rf $O/pmc $O/prof
step prof 240 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --steps 20 --warmup 10 --no-cpu-baseline
step pmc_fetch 120 rocprofv3 --pmc FETCH_SIZE -d $O/pmc/p1 -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline
step pmc_write 120 rocprofv3 --pmc WRITE_SIZE -d $O/pmc/p2 -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline
step pmc_sq 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $O/pmc/p3 -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline
step torchrun1 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 1 --steps 10 --warmup 5 --no-cpu-baseline
exit 0
