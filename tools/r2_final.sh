#!/bin/bash
# Round-2 evidence on the GPU box: full GPU tests, c3 (default) / c2 / c5 bench lines, c3 kernel
# stats, attention PMC traffic (FETCH_SIZE and WRITE_SIZE in separate passes)
set -e
export TMPDIR=/tmp
O=gpurun_out/final
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 500 --timeout-method thread > $O/tests.log 2>&1
timeout -k 10 400 python -u bench.py > $O/bench_c3.log 2>&1
timeout -k 10 300 python -u bench.py --batch 1 --lc 160 --prefix 0 --new-tokens 861 --steps 3 > $O/bench_c2.log 2>&1
timeout -k 10 400 python -u bench.py --model hybrid > $O/bench_c5.log 2>&1
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline > $O/prof.log 2>&1
find $O/prof -type f ! -name "*stats.csv" -delete
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $O/pmc_f -o run --output-format csv -- python3 tools/attn_pmc.py > $O/pmc_f.log 2>&1
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $O/pmc_w -o run --output-format csv -- python3 tools/attn_pmc.py > $O/pmc_w.log 2>&1
python tools/pmc_summary.py $O/pmc_f $O/pmc_w --json $O/attn_pmc.json --match "k_attn_decode<true" --R 128 --ctx 1705 --alg 454033408 > $O/attn_pmc.txt 2>&1
find $O/pmc_f $O/pmc_w -name "*.csv" -size +5M -delete
du -sh $O
