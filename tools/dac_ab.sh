#!/bin/bash
# DAC A/B: product vs zonos_amd/lib/variants/*: per-shape conv timing (tools/dac_layers.py), alternating
set -e
for i in 1 2; do
  echo "== product"; timeout -k 10 180 python tools/dac_layers.py 16 2589 2>&1 | grep -v amdgpu | head -8
  for v in $(ls zonos_amd/lib/variants); do
    echo "== $v"; ZK_LIB_PATH=zonos_amd/lib/variants/$v/libzonos_hip.so timeout -k 10 180 python tools/dac_layers.py 16 2589 2>&1 | grep -v amdgpu | head -8
  done
done
