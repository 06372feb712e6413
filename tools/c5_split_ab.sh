#!/bin/bash
# c5 decode step vs the Mamba in_proj / out_proj split-K counts (ZK_SPLITS overrides)
set -e
export TMPDIR=/tmp
run() { echo "== $1"; ZK_SPLITS="$1" timeout -k 10 400 python bench.py --model hybrid --steps 1 --warmup 1 --no-dac --no-cpu-baseline 2>&1 | grep '^{' | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['breakdown']['decode_ms_per_token_step'])"; }
for i in 1 2; do for sp in "$@"; do run "$sp"; done; done
