#!/bin/bash
# resid_ln standalone timing; c3 split-K retune after the XCD tile order; B=1 heads GEMV layouts
set -e
export TMPDIR=/tmp
O=gpurun_out/sweep
mkdir -p $O
: > $O/out.txt
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_ops.py -k "resid or layernorm or ln" > $O/t.log 2>&1
tail -n 2 $O/t.log >> $O/out.txt
timeout -k 10 120 python tools/microbench.py ln 2>&1 | grep -v amdgpu >> $O/out.txt
for lay in 1 2; do
  echo "== heads layout $lay" >> $O/out.txt
  ZK_GF_LAYOUT=$lay ZK_MB_M=2 ZK_MB_SHAPES=heads:9234:2048:0:1 timeout -k 10 120 python tools/microbench.py gemv 2>&1 | grep "gemv heads" >> $O/out.txt
done
run() { ZK_SPLITS="$1" timeout -k 10 300 python bench.py --steps 1 --warmup 1 --no-dac --no-cpu-baseline 2>&1 | grep '^{' | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('splits=[$1]', d['breakdown']['decode_ms_per_token_step'])" >> $O/out.txt; }
for i in 1 2; do for sp in "" "o=8" "qkv=8" "fc2=16" "o=8,qkv=8"; do run "$sp"; done; done
cat $O/out.txt
