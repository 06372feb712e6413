#!/bin/bash
# A/B of the product library against lib/variants/<name> on the decode GEMM shapes (GPU box).
set -e
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ops.py -k "gemm or swiglu" 2>&1 | tail -1
for i in 1 2; do
  echo "== product"; timeout -k 10 120 python tools/microbench.py gemm 2>&1 | grep gemm
  for v in $(ls zonos_amd/lib/variants); do
    echo "== $v"; ZK_LIB_PATH=zonos_amd/lib/variants/$v/libzonos_hip.so timeout -k 10 120 python tools/microbench.py gemm 2>&1 | grep gemm
  done
done
