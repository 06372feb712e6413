#!/bin/bash
# GPU tests (full suite), c3 bench line + kernel stats, 2-rank rehearsal of the multi-GPU bench path on one GPU
set -e
export TMPDIR=/tmp
O=gpurun_out/r2s3
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 500 --timeout-method thread > $O/tests.log 2>&1
timeout -k 10 400 python -u bench.py > $O/bench.log 2>&1
ZK_BENCH_SHARE_GPU=1 timeout -k 10 400 python -u bench.py --gpus 2 --batch 8 --new-tokens 400 --steps 1 --warmup 1 --no-cpu-baseline > $O/bench_2rank.log 2>&1
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline > $O/prof.log 2>&1
find $O/prof -type f ! -name "*stats.csv" -delete
