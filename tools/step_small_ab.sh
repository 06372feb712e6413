#!/bin/bash
# persistent step anatomy for the product library and each lib/variants/<name> build
set -e
export TMPDIR=/tmp
O=gpurun_out/ss
mkdir -p $O
echo "== product" > $O/ab.txt
timeout -k 10 300 python -u tools/step_small_prof.py 600 2>&1 | grep -v amdgpu.ids >> $O/ab.txt
for v in $(ls zonos_amd/lib/variants); do
  echo "== $v" >> $O/ab.txt
  ZK_LIB_PATH=zonos_amd/lib/variants/$v/libzonos_hip.so timeout -k 10 300 python -u tools/step_small_prof.py 600 2>&1 | grep -v amdgpu.ids >> $O/ab.txt
done
