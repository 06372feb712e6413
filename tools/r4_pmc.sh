#!/bin/bash
# HBM bytes per launch (rocprofv3 PMC, FETCH_SIZE and WRITE_SIZE in separate passes) of the decode
# attention (c3 shape, tools/attn_pmc.py) and the hybrid SSM step (c5 shape, microbench mamba):
#   tools/r4_pmc.sh OUT ROUND   -> profiles-ready summaries in gpurun_out/OUT/
set -e
export TMPDIR=/tmp
OUT=gpurun_out/$1
R=$2
mkdir -p $OUT
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $c -d $OUT/attn_$c -o run --output-format csv -- python3 tools/attn_pmc.py > $OUT/attn_$c.log 2>&1
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $c -d $OUT/mamba_$c -o run --output-format csv -- python3 tools/microbench.py mamba > $OUT/mamba_$c.log 2>&1
done
python tools/pmc_summary.py $OUT/attn_FETCH_SIZE $OUT/attn_WRITE_SIZE --match "k_attn_decode<true" --R 128 --ctx 1705 \
    --alg 454033408 --json $OUT/${R}_attn_fused_pmc.json > $OUT/${R}_attn_fused_pmc.txt
python tools/pmc_summary.py $OUT/mamba_FETCH_SIZE $OUT/mamba_WRITE_SIZE --match "k_mamba_step" --R 128 --ctx 0 \
    --alg 288161792 --json $OUT/${R}_mamba_step_pmc.json > $OUT/${R}_mamba_step_pmc.txt
find $OUT -name "*.csv" -delete
cat $OUT/${R}_attn_fused_pmc.json $OUT/${R}_mamba_step_pmc.json
