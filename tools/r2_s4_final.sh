#!/bin/bash
# Round-2 session-4 evidence: full GPU tests, c3 (default) / c2 / c5 bench lines, c3 and c2 kernel stats
set -e
export TMPDIR=/tmp
O=gpurun_out/s4final6
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 500 --timeout-method thread > $O/tests.log 2>&1
timeout -k 10 500 python -u bench.py > $O/bench_c3.log 2>&1
timeout -k 10 300 python -u bench.py --batch 1 --lc 160 --prefix 0 --new-tokens 861 --steps 3 > $O/bench_c2.log 2>&1
timeout -k 10 500 python -u bench.py --model hybrid > $O/bench_c5.log 2>&1
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline > $O/prof.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof2 -o run -- python3 bench.py --batch 1 --lc 160 --prefix 0 --new-tokens 861 --steps 2 --no-cpu-baseline > $O/prof2.log 2>&1
find $O/prof $O/prof2 -type f ! -name "*stats.csv" -delete
du -sh $O
