#!/bin/bash
# c2 A/B: GEMV tests + c2 bench (product) + ops micro (gemv) 
set -e
export TMPDIR=/tmp
O=gpurun_out/c2q
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_ops.py tests/test_gpu_generate.py tests/test_gpu_fullwidth.py -k "gemv or gemm or swiglu or c1 or c2 or free_running or shard" > $O/t.log 2>&1
for i in 1 2; do timeout -k 10 300 python -u bench.py --batch 1 --lc 160 --prefix 0 --new-tokens 861 --steps 2 --no-cpu-baseline > $O/bench_c2_$i.log 2>&1; done
