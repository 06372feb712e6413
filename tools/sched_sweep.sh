#!/bin/bash
# decode schedule variants at the c3 workload (GPU box): generate-only bench lines.
set -e
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_generate.py -k "two_stream or graph_equals" 2>&1 | tail -1
run() { echo "== $1"; shift; env "$@" timeout -k 10 300 python bench.py --steps 1 --warmup 1 --no-dac --no-cpu-baseline 2>&1 | grep '^{' | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['value'], d['breakdown'].get('decode_ms_per_token_step'))"; }
run base ZK_X=0
run two_stream ZK_TWO_STREAM=1
run two_stream_heads1 ZK_TWO_STREAM=1 ZK_SPLITS=heads=1
