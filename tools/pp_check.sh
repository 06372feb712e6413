#!/bin/bash
# SSM state ping-pong: hybrid tests, mamba microbench, c5 bench
set -e
export TMPDIR=/tmp
O=gpurun_out/pp
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 500 --timeout-method thread tests/test_gpu_hybrid.py > $O/t.log 2>&1
tail -n 2 $O/t.log > $O/out.txt
for i in 1 2; do timeout -k 10 120 python tools/microbench.py mamba 2>&1 | grep mamba_step >> $O/out.txt; done
timeout -k 10 500 python -u bench.py --model hybrid > $O/bench_c5.log 2>&1
python -c "import json; d=json.loads([x for x in open('$O/bench_c5.log') if x.startswith('{')][-1]); print('c5', d['value'], d['rtf'], d['breakdown'], d['roofline']['achieved'], d['roofline']['us_per_launch'])" >> $O/out.txt
cat $O/out.txt
