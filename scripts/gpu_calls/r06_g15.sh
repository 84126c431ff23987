#!/bin/bash
# Round 6, GPU call 15: wgrad_c6 (the nsc backward's dW reductions with every value split once per
# workgroup; the kernel was removed after this A/B) — reduction and training tests, then the config-3
# NLL step A/B against wgrad_x6 (NAZ_WGRAD_C6=0), interleaved, and a kernel trace of the c6 step.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
T=${TAG:-r06_g15}
O=gpurun_out/$T
scripts/gpu_steps.sh $T \
  "wgrad_tests|300|python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_grad.py -k wgrad" \
  "train_tests|900|python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_gpu_train.py" \
  "c6_1|200|python bench.py --train --no-cpu-baseline" \
  "x6_1|200|NAZ_WGRAD_C6=0 python bench.py --train --no-cpu-baseline" \
  "c6_2|200|python bench.py --train --no-cpu-baseline" \
  "x6_2|200|NAZ_WGRAD_C6=0 python bench.py --train --no-cpu-baseline" \
  "kt_c6|300|rocprofv3 --kernel-trace --stats -d $O/kt_c6 -o run --output-format csv -- python3 bench.py --train --no-cpu-baseline --steps 2 --warmup 1"
