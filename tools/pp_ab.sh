#!/bin/bash
# c5: SSM state double-buffered (product) vs in place (ZK_SSM_INPLACE=1), same box, alternating
set -e
export TMPDIR=/tmp
O=gpurun_out/ppab
mkdir -p $O
: > $O/ab.txt
for r in 1 2; do
  for v in 0 1; do
    ZK_SSM_INPLACE=$v timeout -k 10 400 python -u bench.py --model hybrid --steps 1 --warmup 1 --no-dac > $O/b.log 2>&1
    python -c "import json; d=json.loads([x for x in open('$O/b.log') if x.startswith('{')][-1]); print('inplace=$v c5 decode ms', d['breakdown']['decode_ms_per_token_step'], 'mamba us', d['roofline']['us_per_launch'])" >> $O/ab.txt
  done
done
cat $O/ab.txt
