#!/bin/bash
# persistent small-batch step: bit-identity vs the launch sequence, full-width parity, c2 bench
set -e
export TMPDIR=/tmp
O=gpurun_out/ss
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_step_small.py -x -v -s --timeout 500 --timeout-method thread > $O/t_step.log 2>&1
timeout -k 10 400 python -u -m pytest tests/test_gpu_fullwidth.py -x -v -k "c1 or c2" --timeout 300 --timeout-method thread > $O/t_full.log 2>&1
timeout -k 10 300 python -u bench.py --batch 1 --lc 160 --prefix 0 --new-tokens 861 --steps 2 --no-cpu-baseline > $O/bench_c2.log 2>&1
ZK_PERSIST=0 timeout -k 10 300 python -u bench.py --batch 1 --lc 160 --prefix 0 --new-tokens 861 --steps 2 --no-cpu-baseline > $O/bench_c2_launch.log 2>&1
