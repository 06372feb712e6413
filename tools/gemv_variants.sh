#!/bin/bash
# Small-batch GEMV tuning on the GPU box: default build + build_variant libraries (tools/gemv_variants.py)
set -e
export TMPDIR=/tmp
for v in default $(ls zonos_amd/lib/variants 2>/dev/null); do
  if [ "$v" = default ]; then unset ZK_LIB_PATH; else export ZK_LIB_PATH=zonos_amd/lib/variants/$v/libzonos_hip.so; fi
  echo "== $v"
  for m in ${MS:-2 16}; do ZK_MB_M=$m timeout -k 10 120 python tools/microbench.py gemv 2>&1 | grep -v amdgpu.ids; done
done
