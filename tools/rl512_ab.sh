#!/bin/bash
# k_resid_ln: 512-thread rows (ZK_RL512=1) vs 256 (product); LN tests under the knob; c3 decode step
set -e
export TMPDIR=/tmp
O=gpurun_out/rl512
mkdir -p $O
ZK_RL512=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_ops.py -k "resid or layernorm or ln" > $O/t.log 2>&1
tail -n 1 $O/t.log > $O/ab.txt
for r in 1 2; do
  for v in 0 1; do
    ZK_RL512=$v timeout -k 10 120 python tools/microbench.py ln 2>&1 | grep "rows=128" | sed "s/^/rl512=$v /" >> $O/ab.txt
    ZK_RL512=$v timeout -k 10 300 python -u bench.py --steps 1 --warmup 1 --no-dac --no-cpu-baseline > $O/b.log 2>&1
    python -c "import json; d=json.loads([x for x in open('$O/b.log') if x.startswith('{')][-1]); print('rl512=$v c3 decode ms', d['breakdown']['decode_ms_per_token_step'])" >> $O/ab.txt
  done
done
cat $O/ab.txt
