#!/bin/bash
# decode GEMMs at M=128: one 128-row workgroup per column tile vs two 64-row twins (ZK_WS_HALVES=1)
set -e
export TMPDIR=/tmp
O=gpurun_out/halves
mkdir -p $O
ZK_WS_HALVES=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_ops.py -k "gemm" > $O/t.log 2>&1
ZK_WS_HALVES=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_fullwidth.py -k "c3" >> $O/t.log 2>&1
: > $O/ab.txt
for r in 1 2; do
  for h in 0 1; do echo "== halves $h" >> $O/ab.txt; ZK_WS_HALVES=$h timeout -k 10 120 python tools/microbench.py gemm 2>&1 | grep gemm >> $O/ab.txt; done
done
for r in 1 2; do
  for h in 0 1; do
    ZK_WS_HALVES=$h timeout -k 10 300 python -u bench.py --steps 1 --warmup 1 --no-dac --no-cpu-baseline > $O/b.log 2>&1
    python -c "import json; d=json.loads([x for x in open('$O/b.log') if x.startswith('{')][-1]); print('bench halves $h', d['breakdown']['decode_ms_per_token_step'])" >> $O/ab.txt
  done
done
cat $O/ab.txt
