#!/bin/bash
# DAC residual stream double-buffered (product) vs in place (ZK_DAC_INPLACE=1)
set -e
export TMPDIR=/tmp
O=gpurun_out/dacpp
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_dac.py tests/test_gpu_dac_cl.py > $O/t.log 2>&1
tail -n 2 $O/t.log > $O/ab.txt
for r in 1 2; do
  for v in 0 1; do
    echo "== inplace=$v" >> $O/ab.txt
    ZK_DAC_INPLACE=$v timeout -k 10 180 python tools/dac_layers.py 16 2589 2>&1 | grep -v amdgpu | head -8 >> $O/ab.txt
  done
done
cat $O/ab.txt
