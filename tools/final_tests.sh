#!/bin/bash
set -e
export TMPDIR=/tmp
O=gpurun_out/ft
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 500 --timeout-method thread > $O/tests.log 2>&1
tail -n 1 $O/tests.log
timeout -k 10 300 python -u bench.py --steps 1 --warmup 1 --no-dac --no-cpu-baseline > $O/b.log 2>&1
python -c "import json; d=json.loads([x for x in open('$O/b.log') if x.startswith('{')][-1]); print('c3 decode ms', d['breakdown']['decode_ms_per_token_step'])"
