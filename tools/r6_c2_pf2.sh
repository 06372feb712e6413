#!/bin/bash
# round 6 c2: k-steps in flight of the B = 1 GEMVs (ZK_GF_PF2 / ZK_GF_PFLN) after the LDS-staged activation:
# product (8 / 12) against pf4 (4 / 12), pf6 (6 / 12), pfln8 (8 / 8), interleaved
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
for i in 1 2 3; do
  for v in product pf4 pf6 pfln8; do
    lp=""; [ "$v" != product ] && lp=zonos_amd/lib/variants/$v/libzonos_hip.so
    ZK_LIB_PATH=$lp ZK_C2_REPS=2 timeout -k 10 300 python -u tools/c2_step.py 4 > $O/c2_$v.log 2>&1 || exit 1
    grep "^c2" $O/c2_$v.log | sed "s/^/$v /"
  done
done
