#!/bin/bash
# decode-step A/B of split-K choices (ZK_SPLITS overrides), same box, alternating (GPU box)
set -e
run() { echo "== $1"; ZK_SPLITS="$1" timeout -k 10 300 python bench.py --steps 1 --warmup 1 --no-dac --no-cpu-baseline 2>&1 | grep '^{' | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['breakdown']['decode_ms_per_token_step'])"; }
for i in 1 2; do for sp in "$@"; do run "$sp"; done; done
