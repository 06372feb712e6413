#!/bin/bash
# round 6 c3: decode attention key splits (1 = product, 2 / 4 with the in-launch combine), interleaved
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
A="--steps 2 --warmup 1 --no-secondary --no-cpu-baseline"
for i in 1 2; do
  for n in 1 2 4; do
    timeout -k 10 300 python -u tools/c3_splits.py $n $A > $O/c3_s$n.log 2>&1 || exit 1
    grep '^{' $O/c3_s$n.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('splits $n', d['value'], d['breakdown']['decode_ms_per_token_step'])"
  done
done
