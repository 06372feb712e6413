#!/bin/bash
# k_mamba_step per-head vs grouped variants (tools/microbench.py mamba), two alternating passes
export TMPDIR=/tmp
for r in 1 2; do
  unset ZK_LIB_PATH
  ZK_MAMBA_GROUPED=0 timeout -k 10 60 python tools/microbench.py mamba 2>&1 | grep -v amdgpu.ids
  for v in default $(ls zonos_amd/lib/variants); do
    if [ $v = default ]; then unset ZK_LIB_PATH; else export ZK_LIB_PATH=zonos_amd/lib/variants/$v/libzonos_hip.so; fi
    echo -n "$v: "; timeout -k 10 60 python tools/microbench.py mamba 2>&1 | grep -v amdgpu.ids
  done
done
