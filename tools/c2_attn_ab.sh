#!/bin/bash
# B=1 decode (c2): attention key-split count A/B (GPU box)
set -e
for sp in "" 1 2 4; do
  echo "== ZK_ATTN_SPLITS=$sp"
  ZK_ATTN_SPLITS=$sp timeout -k 10 300 python bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-dac --batch 1 --lc 160 --prefix 0 --new-tokens 861 2>&1 | grep '^{' | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['breakdown']['decode_ms_per_token_step'])"
done
