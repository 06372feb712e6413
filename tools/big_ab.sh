#!/bin/bash
# A/B of the 256 x 128-tile prefill GEMM against the 128 x 64 one (tools/microbench.py prefill)
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q --timeout 120 --timeout-method thread \
    -k "gemm or swiglu" > gpurun_out/big_tests.log 2>&1
for i in 1 2; do
  ZK_BIG_GEMM=0 timeout -k 10 120 python -u tools/microbench.py prefill > gpurun_out/big_off_$i.log 2>&1
  ZK_BIG_GEMM=1 timeout -k 10 120 python -u tools/microbench.py prefill > gpurun_out/big_on_$i.log 2>&1
done
tail -n 3 gpurun_out/big_tests.log
grep -H prefill gpurun_out/big_o*.log
