#!/bin/bash
# round 2, first GPU call: suite + headline bench + training bench (strong, 2^23 global on 1 GPU)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r02_pytest.log 2>&1 || { tail -30 gpurun_out/r02_pytest.log; exit 1; }
tail -2 gpurun_out/r02_pytest.log
timeout -k 10 180 python bench.py > gpurun_out/r02_bench.json 2> gpurun_out/r02_bench.err || { cat gpurun_out/r02_bench.err | tail -20; exit 1; }
cat gpurun_out/r02_bench.json
timeout -k 10 300 python bench.py --train --steps 5 --warmup 2 > gpurun_out/r02_train.json 2> gpurun_out/r02_train.err || { tail -20 gpurun_out/r02_train.err; exit 1; }
cat gpurun_out/r02_train.json
