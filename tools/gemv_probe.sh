#!/bin/bash
# small-batch GEMV: layouts x variants at the c2 shapes (M=2) and M=16
export TMPDIR=/tmp
for lib in default $(ls zonos_amd/lib/variants 2>/dev/null); do
  if [ $lib = default ]; then unset ZK_LIB_PATH; else export ZK_LIB_PATH=zonos_amd/lib/variants/$lib/libzonos_hip.so; fi
  for lay in ${LAYS:--1 0 1}; do
    echo "== lib $lib layout $lay"
    for m in ${MS:-2}; do
      ZK_GF_LAYOUT=$lay ZK_MB_M=$m timeout -k 10 120 python tools/microbench.py gemv 2>&1 | grep -v amdgpu.ids
    done
  done
done
