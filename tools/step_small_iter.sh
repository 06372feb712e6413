#!/bin/bash
# persistent small-batch step: bit-identity test + phase anatomy + c2 bench line
set -e
export TMPDIR=/tmp
O=gpurun_out/ss
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_step_small.py -x -v -s --timeout 500 --timeout-method thread > $O/t_step.log 2>&1
timeout -k 10 300 python -u tools/step_small_prof.py 600 > $O/prof600.txt 2>&1
timeout -k 10 300 python -u bench.py --batch 1 --lc 160 --prefix 0 --new-tokens 861 --steps 2 --no-cpu-baseline > $O/bench_c2.log 2>&1
