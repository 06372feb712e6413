#!/bin/bash
# k_gemm_ws epilogue: LDS-staged whole-row stores (default) vs direct fragment stores (variant epi0)
export TMPDIR=/tmp
for r in 1 2; do
  for v in default epi0; do
    if [ $v = default ]; then unset ZK_LIB_PATH; else export ZK_LIB_PATH=zonos_amd/lib/variants/$v/libzonos_hip.so; fi
    echo "== $v"; ZK_MB_M=128 timeout -k 10 120 python tools/microbench.py gemm 2>&1 | grep -v amdgpu.ids
  done
done
unset ZK_LIB_PATH
