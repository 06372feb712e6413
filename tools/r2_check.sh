#!/bin/bash
# Session check on the GPU box: GPU tests, default (c3) bench line, kernel stats of one bench step.
set -e
export TMPDIR=/tmp
O=gpurun_out/r2chk
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1
timeout -k 10 400 python -u bench.py > $O/bench.log 2>&1
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline > $O/prof.log 2>&1
find $O/prof -type f ! -name "*stats.csv" -delete
du -sh $O
