#!/bin/bash
# c2 (B=1) decode step: attention key splits merged in the out_proj GEMV prologue (ZK_ATTN_MERGE)
set -e
export TMPDIR=/tmp
O=gpurun_out/merge
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_ops.py -k "merge or attention or gemv" > $O/t.log 2>&1
: > $O/ab.txt
for r in 1 2; do
  for n in 0 2 4 8; do
    ZK_ATTN_MERGE=$n timeout -k 10 300 python -u bench.py --batch 1 --lc 160 --prefix 0 --new-tokens 861 --steps 2 --no-dac --no-cpu-baseline > $O/b.log 2>&1
    python -c "import json; d=json.loads([x for x in open('$O/b.log') if x.startswith('{')][-1]); print('merge=$n c2 decode ms', d['breakdown']['decode_ms_per_token_step'])" >> $O/ab.txt
  done
done
cat $O/ab.txt
