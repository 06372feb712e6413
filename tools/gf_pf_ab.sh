#!/bin/bash
# k_gemv_f weight loads in flight per wave (ZK_GF_PF): product (8) vs variants, microbench + c2 step
set -e
export TMPDIR=/tmp
O=gpurun_out/gfpf
mkdir -p $O
: > $O/ab.txt
for r in 1 2; do
  for v in product $(ls zonos_amd/lib/variants); do
    lp=""; [ "$v" != product ] && lp=zonos_amd/lib/variants/$v/libzonos_hip.so
    echo "== $v" >> $O/ab.txt
    ZK_LIB_PATH=$lp ZK_MB_M=2 timeout -k 10 200 python tools/microbench.py gemv 2>&1 | grep -v amdgpu >> $O/ab.txt
  done
done
for r in 1 2; do
  for v in product $(ls zonos_amd/lib/variants); do
    lp=""; [ "$v" != product ] && lp=zonos_amd/lib/variants/$v/libzonos_hip.so
    ZK_LIB_PATH=$lp timeout -k 10 300 python -u bench.py --batch 1 --lc 160 --prefix 0 --new-tokens 861 --steps 2 --no-dac --no-cpu-baseline > $O/b.log 2>&1
    python -c "import json; d=json.loads([x for x in open('$O/b.log') if x.startswith('{')][-1]); print('$v c2 decode ms', d['breakdown']['decode_ms_per_token_step'])" >> $O/ab.txt
  done
done
cat $O/ab.txt
