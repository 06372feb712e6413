#!/bin/bash
# round 6 c5: Mamba in_proj split-K 1 (product) / 2 / 4 after the step-word change, interleaved
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
A="--model hybrid --steps 1 --warmup 1 --no-secondary --no-cpu-baseline"
for i in 1 2; do
  for n in 1 2 4; do
    timeout -k 10 300 python -u tools/c5_inp.py $n $A > $O/c5_s$n.log 2>&1 || exit 1
    grep '^{' $O/c5_s$n.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('inp split $n', d['value'], d['breakdown']['decode_ms_per_token_step'])"
  done
done
