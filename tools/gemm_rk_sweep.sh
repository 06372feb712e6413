#!/bin/bash
# decode-GEMM kernel forms at the decode shapes (GPU box). Correctness first.
set -e
for k in ws3 rk; do
  ZK_GEMM_KERNEL=$k timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ops.py -k "gemm or swiglu" 2>&1 | tail -1
done
echo "== ws (loader-wave form)"; ZK_GEMM_KERNEL=ws timeout -k 10 120 python tools/microbench.py gemm 2>&1 | grep gemm
echo "== ws3"; ZK_GEMM_KERNEL=ws3 timeout -k 10 120 python tools/microbench.py gemm 2>&1 | grep gemm
for sp in "qkv=2,o=4,fc2=4,heads=1" "qkv=8,o=16,fc2=16,heads=4"; do
  echo "== ws3 splits $sp"; ZK_GEMM_KERNEL=ws3 ZK_SPLITS=$sp timeout -k 10 120 python tools/microbench.py gemm 2>&1 | grep gemm
  echo "== ws splits $sp"; ZK_GEMM_KERNEL=ws ZK_SPLITS=$sp timeout -k 10 120 python tools/microbench.py gemm 2>&1 | grep gemm
done
