#!/bin/bash
# zk_dac_decode (whole DAC decode through the C ABI) vs the Python sequence; DAC tests; c3 DAC time
set -e
export TMPDIR=/tmp
O=gpurun_out/cdac
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 500 --timeout-method thread tests/test_gpu_dac.py tests/test_gpu_dropin.py > $O/t1.log 2>&1
: > $O/ab.txt
for v in 1 0; do
  ZK_C_DAC=$v timeout -k 10 400 python -u bench.py --steps 1 --warmup 1 --no-cpu-baseline > $O/b.log 2>&1
  python -c "import json; d=json.loads([x for x in open('$O/b.log') if x.startswith('{')][-1]); print('c_dac=$v c3', d['value'], d['breakdown']['dac_s_per_step'])" >> $O/ab.txt
done
grep -E "PASSED|FAILED" $O/t1.log | tail -30
cat $O/ab.txt
