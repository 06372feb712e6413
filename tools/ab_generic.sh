#!/bin/bash
# A/B of the product library vs lib/variants/<name>: microbench mode $1 (+ optional decode bench)
set -e
for i in 1 2; do
  echo "== product"; timeout -k 10 120 python tools/microbench.py $1 2>&1 | grep -v amdgpu
  for v in $(ls zonos_amd/lib/variants); do
    echo "== $v"; ZK_LIB_PATH=zonos_amd/lib/variants/$v/libzonos_hip.so timeout -k 10 120 python tools/microbench.py $1 2>&1 | grep -v amdgpu
  done
done
if [ -n "$BENCH" ]; then
  for v in product $(ls zonos_amd/lib/variants); do
    lp=""; [ "$v" != product ] && lp=zonos_amd/lib/variants/$v/libzonos_hip.so
    echo "== bench $v"; ZK_LIB_PATH=$lp timeout -k 10 300 python bench.py --steps 1 --warmup 1 --no-dac --no-cpu-baseline 2>&1 | grep '^{' | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['breakdown']['decode_ms_per_token_step'])"
  done
fi
