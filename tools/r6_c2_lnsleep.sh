#!/bin/bash
# round 6 c2: B = 1 LayerNorm GEMVs sleeping 64*N clocks before their weight prefetch (lnsleepN, ZK_GF_LNSLEEP) and 16 k-steps in flight for the in_proj (pfln16) vs product; ms per c2 decode step
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
for i in 1 2; do
  for v in product lnsleep8 lnsleep16 lnsleep32 pfln16; do
    lp=""; [ "$v" != product ] && lp=zonos_amd/lib/variants/$v/libzonos_hip.so
    ZK_LIB_PATH=$lp ZK_C2_REPS=2 timeout -k 10 300 python -u tools/c2_step.py 4 > $O/c2_$v.log 2>&1 || exit 1
    grep "^c2" $O/c2_$v.log | sed "s/^/$v /"
  done
done
