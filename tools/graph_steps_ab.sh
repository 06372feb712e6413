#!/bin/bash
# decode steps per hipGraph replay: 1 vs 4 (and 8), c2 and c3 decode steps
set -e
export TMPDIR=/tmp
O=gpurun_out/gs
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_generate.py tests/test_gpu_fullwidth.py tests/test_gpu_dropin.py > $O/t.log 2>&1
: > $O/ab.txt
for r in 1 2; do
  for k in 1 4 8; do
    ZK_GRAPH_STEPS=$k timeout -k 10 300 python -u bench.py --batch 1 --lc 160 --prefix 0 --new-tokens 861 --steps 2 --no-dac --no-cpu-baseline > $O/b.log 2>&1
    python -c "import json; d=json.loads([x for x in open('$O/b.log') if x.startswith('{')][-1]); print('steps/graph $k c2 decode ms', d['breakdown']['decode_ms_per_token_step'])" >> $O/ab.txt
  done
done
for k in 1 4; do
  ZK_GRAPH_STEPS=$k timeout -k 10 300 python -u bench.py --steps 1 --warmup 1 --no-dac --no-cpu-baseline > $O/b.log 2>&1
  python -c "import json; d=json.loads([x for x in open('$O/b.log') if x.startswith('{')][-1]); print('steps/graph $k c3 decode ms', d['breakdown']['decode_ms_per_token_step'])" >> $O/ab.txt
done
cat $O/ab.txt
