#!/bin/bash
# DAC per-layer timing, product vs lib/variants/* (GPU box)
set -e
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_dac_cl.py tests/test_gpu_dac.py tests/test_gpu_dac_enc.py 2>&1 | tail -1
for v in product $(ls zonos_amd/lib/variants); do
  lp=""; [ "$v" != product ] && lp=zonos_amd/lib/variants/$v/libzonos_hip.so
  echo "== $v"; ZK_LIB_PATH=$lp timeout -k 10 300 python tools/dac_layers.py 16 2589 2>&1 | grep -v amdgpu
done
