#!/bin/bash
# Round 6 final GPU call: smoke, the whole GPU suite, the headline bench and its kernel trace, fresh
# HBM-traffic PMC passes of the headline kernel, the configs[1] line, the AR lines (nsa16 / maf), the
# config-3 NLL step (with its CPU baseline) and its kernel trace, the wide-maf NLL step (2^16 rows,
# naz's 10,752-row minibatch eager and graphed), CNF log_prob and CNF training.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
T=${TAG:-r06_final}
P=gpurun_out/$T
RP="rocprofv3 --kernel-trace --stats -o run --output-format csv"
TR="python bench.py --train --flow maf4 --no-cpu-baseline"
scripts/gpu_steps.sh $T \
  "smoke|300|python -c 'import __graft_entry__ as g; g.smoke()'" \
  "tests|900|python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider" \
  "bench|300|python bench.py" \
  "prof_bench|240|$RP -d $P/prof_bench -- python3 bench.py --steps 20 --warmup 10 --no-cpu-baseline" \
  "pmc_fetch|120|rocprofv3 --pmc FETCH_SIZE -d $P/pmc_fetch -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline" \
  "pmc_write|120|rocprofv3 --pmc WRITE_SIZE -d $P/pmc_write -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline" \
  "config2|300|python bench.py --flow config2" \
  "nsa16|200|python bench.py --flow nsa16 --no-cpu-baseline --steps 30" \
  "maf|200|python bench.py --flow maf --no-cpu-baseline --steps 30" \
  "train|400|python bench.py --train" \
  "prof_train|300|$RP -d $P/prof_train -- python3 bench.py --train --no-cpu-baseline --steps 3 --warmup 1" \
  "maf4|300|$TR --steps 5 --warmup 2" \
  "maf4_nb|300|$TR --batch 10752 --steps 10 --warmup 3" \
  "maf4_nb_graph|300|$TR --batch 10752 --steps 10 --warmup 3 --graph" \
  "cnf|300|python bench.py --cnf --no-cpu-baseline" \
  "cnf_train|300|python bench.py --cnf-train --no-cpu-baseline --steps 5 --warmup 2"
