#!/bin/bash
# DAC k7 convs: deep form (one workgroup per CU, 256 positions, 8 weight slices in flight; ZK_DAC_DEEP=1) vs default
set -e
export TMPDIR=/tmp
O=gpurun_out/deep
mkdir -p $O
ZK_DAC_DEEP=1 timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_dac.py tests/test_gpu_dac_cl.py > $O/t.log 2>&1
tail -n 2 $O/t.log > $O/ab.txt
for r in 1 2; do
  for d in 0 1; do
    echo "== deep=$d" >> $O/ab.txt
    ZK_DAC_DEEP=$d timeout -k 10 180 python tools/dac_layers.py 16 2589 2>&1 | grep -v amdgpu >> $O/ab.txt
  done
done
for d in 0 1; do
  ZK_DAC_DEEP=$d timeout -k 10 400 python -u bench.py --steps 1 --warmup 1 --no-cpu-baseline > $O/b.log 2>&1
  python -c "import json; d=json.loads([x for x in open('$O/b.log') if x.startswith('{')][-1]); print('deep=$d c3', d['value'], d['breakdown'])" >> $O/ab.txt
done
cat $O/ab.txt
