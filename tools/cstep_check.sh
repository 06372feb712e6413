#!/bin/bash
# zk_decode_step (C ABI step) vs the Python sequence; full GPU tests; c2/c3 decode step timing
set -e
export TMPDIR=/tmp
O=gpurun_out/cstep
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 500 --timeout-method thread tests/test_gpu_generate.py -k "c_decode_step or full_c1 or dropin" > $O/t1.log 2>&1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 500 --timeout-method thread > $O/tests.log 2>&1
: > $O/ab.txt
for v in 1 0; do
  ZK_C_STEP=$v timeout -k 10 300 python -u bench.py --steps 1 --warmup 1 --no-dac --no-cpu-baseline > $O/b.log 2>&1
  python -c "import json; d=json.loads([x for x in open('$O/b.log') if x.startswith('{')][-1]); print('c_step=$v c3 decode ms', d['breakdown']['decode_ms_per_token_step'])" >> $O/ab.txt
  ZK_C_STEP=$v timeout -k 10 300 python -u bench.py --batch 1 --lc 160 --prefix 0 --new-tokens 861 --steps 2 --no-dac --no-cpu-baseline > $O/b.log 2>&1
  python -c "import json; d=json.loads([x for x in open('$O/b.log') if x.startswith('{')][-1]); print('c_step=$v c2 decode ms', d['breakdown']['decode_ms_per_token_step'])" >> $O/ab.txt
done
grep -E "PASSED|FAILED" $O/t1.log
tail -n 1 $O/tests.log
cat $O/ab.txt
