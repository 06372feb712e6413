#!/bin/bash
# round 6 vs round 5 on ONE box: the round-5 tree (commit 87a8e7b, staged in r5tree/ with its own library) and the
# current tree, interleaved, c3 / c2 / c5 -- codes/s and decode ms per step
set -o pipefail
export TMPDIR=/tmp
O=$PWD/gpurun_out/$1
mkdir -p $O
C3="--steps 2 --warmup 1 --no-cpu-baseline"
C2="--batch 1 --lc 160 --prefix 0 --new-tokens 861 --steps 3 --warmup 1 --no-cpu-baseline"
C5="--model hybrid --steps 1 --warmup 1 --no-cpu-baseline"
show() { grep '^{' "$2" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$1', d['value'], d['breakdown'].get('decode_ms_per_token_step'))"; }
for i in 1 2; do
  for cfg in c3 c2 c5; do
    case $cfg in c3) A=$C3;; c2) A=$C2;; c5) A=$C5;; esac
    (cd r5tree && timeout -k 10 300 python -u bench.py $A > $O/r5_$cfg.log 2>&1) || exit 1
    show "r5 $cfg" $O/r5_$cfg.log
    timeout -k 10 300 python -u bench.py $A --no-secondary > $O/r6_$cfg.log 2>&1 || exit 1
    show "r6 $cfg" $O/r6_$cfg.log
  done
done
