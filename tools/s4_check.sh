#!/bin/bash
# full GPU tests on the current tree, then sc1 write-through slab stores (variants/sc1) vs nt (product) at c3
set -e
export TMPDIR=/tmp
O=gpurun_out/s4c
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 500 --timeout-method thread > $O/tests.log 2>&1
: > $O/ab.txt
for r in 1 2; do
  for v in product sc1; do
    lp=""; [ "$v" != product ] && lp=zonos_amd/lib/variants/$v/libzonos_hip.so
    ZK_LIB_PATH=$lp timeout -k 10 300 python -u bench.py --steps 1 --warmup 1 --no-dac --no-cpu-baseline > $O/b.log 2>&1
    python -c "import json; d=json.loads([x for x in open('$O/b.log') if x.startswith('{')][-1]); print('$v c3 decode ms', d['breakdown']['decode_ms_per_token_step'])" >> $O/ab.txt
  done
done
cat $O/ab.txt
