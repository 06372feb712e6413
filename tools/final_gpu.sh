#!/bin/bash
# Round-end evidence on the GPU box: tests, default bench line, kernel stats, PMC traffic.
set -e
export TMPDIR=/tmp
O=gpurun_out/final
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
timeout -k 10 400 python -u bench.py > $O/bench.log 2>&1
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline > $O/prof.log 2>&1
find $O/prof -type f ! -name "*stats.csv" -delete
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $O/pmc_f -o run --output-format csv -- python3 tools/attn_pmc.py > $O/pmc_f.log 2>&1
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $O/pmc_w -o run --output-format csv -- python3 tools/attn_pmc.py > $O/pmc_w.log 2>&1
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $O/gpmc_f -o run --output-format csv -- python3 tools/gemm_pmc.py > $O/gpmc_f.log 2>&1
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $O/gpmc_w -o run --output-format csv -- python3 tools/gemm_pmc.py > $O/gpmc_w.log 2>&1
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE -d $O/dpmc -o run --output-format csv -- python3 tools/dac_pmc.py > $O/dpmc.log 2>&1
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE -d $O/gmpmc -o run --output-format csv -- python3 tools/gemm_pmc.py > $O/gmpmc.log 2>&1
python tools/mfma_summary.py $O/dpmc --match k_conv_cl --json $O/dac_mfma.json > $O/dac_mfma.txt 2>&1
python tools/mfma_summary.py $O/gmpmc --match k_gemm --json $O/gemm_mfma.json > $O/gemm_mfma.txt 2>&1
find $O -name "*.csv" -size +20M -delete
du -sh $O
