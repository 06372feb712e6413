#!/bin/bash
# c2 / c5 bench lines + a c2 kernel trace (per-launch anatomy of the B=1 decode step)
set -e
export TMPDIR=/tmp
O=gpurun_out/c2c5
mkdir -p $O
timeout -k 10 300 python -u bench.py --batch 1 --lc 160 --prefix 0 --new-tokens 861 --steps 3 > $O/bench_c2.log 2>&1
timeout -k 10 400 python -u bench.py --model hybrid > $O/bench_c5.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tr -o run -- python3 bench.py --batch 1 --lc 160 --prefix 0 --new-tokens 300 --steps 1 --warmup 0 --no-cpu-baseline --no-dac > $O/tr.log 2>&1
python tools/trace_step.py $(find $O/tr -name "*kernel_trace.csv") --last 100 --seq > $O/c2_anatomy.txt
find $O/tr -type f -delete
