#!/bin/bash
# B=1 decode (c2) A/B: product vs zonos_amd/lib/variants/* (GPU box), alternating
set -e
for i in 1 2; do
  for v in product $(ls zonos_amd/lib/variants); do
    lp=""; [ "$v" != product ] && lp=zonos_amd/lib/variants/$v/libzonos_hip.so
    echo "== $v $(ZK_LIB_PATH=$lp timeout -k 10 300 python bench.py --steps 1 --warmup 1 --no-dac --no-cpu-baseline --batch 1 --lc 160 --prefix 0 --new-tokens 861 2>&1 | grep '^{' | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['breakdown']['decode_ms_per_token_step'])")"
  done
done
