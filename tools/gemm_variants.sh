#!/bin/bash
# Build decode-GEMM tuning variants (lib/variants/<name>) and time them with tools/microbench.py gemm.
# Usage (GPU box): bash tools/gemm_variants.sh   [variants must be prebuilt: python tools/gemm_variants.py]
set -e
for v in $(ls zonos_amd/lib/variants); do
  echo "== $v"
  ZK_LIB_PATH=zonos_amd/lib/variants/$v/libzonos_hip.so timeout -k 10 120 python tools/microbench.py gemm
  [ -n "$NOTEST" ] || ZK_LIB_PATH=zonos_amd/lib/variants/$v/libzonos_hip.so timeout -k 10 300 python -m pytest -q -x tests/test_gpu_ops.py -k "gemm or swiglu" 2>&1 | tail -1
done
