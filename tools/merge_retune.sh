#!/bin/bash
# c2: attention merge splits 2 / 4 / 8 after the 2-row GEMV image
set -e
export TMPDIR=/tmp
O=gpurun_out/mr
mkdir -p $O
: > $O/ab.txt
for r in 1 2; do
  for n in 4 8 2; do
    ZK_ATTN_MERGE=$n timeout -k 10 300 python -u bench.py --batch 1 --lc 160 --prefix 0 --new-tokens 861 --steps 2 --no-dac --no-cpu-baseline > $O/b.log 2>&1
    python -c "import json; d=json.loads([x for x in open('$O/b.log') if x.startswith('{')][-1]); print('merge=$n c2 decode ms', d['breakdown']['decode_ms_per_token_step'])" >> $O/ab.txt
  done
done
cat $O/ab.txt
