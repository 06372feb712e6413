#!/bin/bash
# c5 (hybrid) decode A/B of alternative libraries against the product, interleaved, twice:
#   tools/r4_c5_ab.sh OUT LIB [LIB ...]
set -e
export TMPDIR=/tmp
OUT=gpurun_out/$1
shift
mkdir -p $OUT
for i in 1 2; do
  for v in product "$@"; do
    lp=""; [ "$v" != product ] && lp=$v
    ZK_LIB_PATH=$lp timeout -k 10 400 python -u bench.py --model hybrid --no-dac --steps 1 --warmup 1 --no-cpu-baseline > $OUT/c5_tmp.log 2>&1
    grep '^{' $OUT/c5_tmp.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); b=d['breakdown']; print('$v', d['value'], b.get('decode_ms_per_token_step'))"
  done
done > $OUT/c5_ab.log 2>&1
rm -f $OUT/c5_tmp.log
cat $OUT/c5_ab.log
