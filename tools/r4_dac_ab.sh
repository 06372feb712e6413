#!/bin/bash
# DAC conv variant A/B: per-layer table + whole decode, product and every variant, then the DAC tests
# on each variant (parity must hold for any SPB / DA).
set -e
export TMPDIR=/tmp
OUT=gpurun_out/$1
mkdir -p $OUT
for i in 1 2; do
  for v in product $(ls zonos_amd/lib/variants); do
    lp=""; [ "$v" != product ] && lp=zonos_amd/lib/variants/$v/libzonos_hip.so
    echo "== $v"; ZK_LIB_PATH=$lp timeout -k 10 240 python tools/microbench.py dac
  done
done > $OUT/dac_micro.log 2>&1
grep -v amdgpu.ids $OUT/dac_micro.log
for v in $(ls zonos_amd/lib/variants); do
  ZK_LIB_PATH=zonos_amd/lib/variants/$v/libzonos_hip.so timeout -k 10 600 python -u -m pytest tests/test_gpu_dac.py tests/test_gpu_dac_cl.py tests/test_gpu_dac_enc.py -x -q --timeout 300 --timeout-method thread > $OUT/tests_$v.log 2>&1
  echo "$v: $(tail -1 $OUT/tests_$v.log)"
done
