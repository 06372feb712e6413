#!/bin/bash
# B=1 decode (c2): small-M GEMV on/off (GPU box)
set -e
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ops.py -k "gemm or swiglu" 2>&1 | tail -1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_generate.py 2>&1 | tail -1
for g in 1 0; do
  echo "== ZK_GEMV=$g"; ZK_GEMV=$g ZK_MB_M=2 timeout -k 10 120 python tools/microbench.py gemm 2>&1 | grep gemm
  ZK_GEMV=$g timeout -k 10 300 python bench.py --steps 1 --warmup 1 --no-cpu-baseline --batch 1 --lc 160 --prefix 0 --new-tokens 861 2>&1 | grep '^{' | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['value'], d['rtf'], d['breakdown'])"
done
