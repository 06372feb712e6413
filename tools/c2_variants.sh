#!/bin/bash
# c2 decode step: product library vs lib/variants/<name> (alternating, 2 rounds)
set -e
export TMPDIR=/tmp
O=gpurun_out/c2v
mkdir -p $O
: > $O/ab.txt
for rnd in 1 2; do
  for v in product $(ls zonos_amd/lib/variants); do
    lp=""; [ "$v" != product ] && lp=zonos_amd/lib/variants/$v/libzonos_hip.so
    ZK_LIB_PATH=$lp timeout -k 10 300 python -u bench.py --batch 1 --lc 160 --prefix 0 --new-tokens 861 --steps 2 --no-cpu-baseline --no-dac > $O/b.log 2>&1
    python -c "import json; d=json.loads([x for x in open('$O/b.log') if x.startswith('{')][-1]); print('$v', d['breakdown']['decode_ms_per_token_step'], d['roofline']['us_per_launch'])" >> $O/ab.txt
  done
done
cat $O/ab.txt
