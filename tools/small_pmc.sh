#!/bin/bash
# PMC traffic of the c2 (k_gemv_f fc1, M = 2) and c5 (k_mamba_step) dominant kernels
set -e
export TMPDIR=/tmp
O=gpurun_out/spmc
mkdir -p $O
for m in gemv mamba; do
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $O/${m}_f -o run --output-format csv -- python3 tools/small_pmc.py $m > $O/${m}_f.log 2>&1
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $O/${m}_w -o run --output-format csv -- python3 tools/small_pmc.py $m > $O/${m}_w.log 2>&1
done
python tools/pmc_summary.py $O/gemv_f $O/gemv_w --json $O/gemv_pmc.json --match "k_gemv_f<1, true" --R 2 --ctx 0 --alg 67158016 --key N=16384 --key K=2048 > $O/gemv_pmc.txt 2>&1
python tools/pmc_summary.py $O/mamba_f $O/mamba_w --json $O/mamba_pmc.json --match "k_mamba_step" --R 128 --ctx 0 --alg 283803648 > $O/mamba_pmc.txt 2>&1
find $O -name "*.csv" -size +5M -delete
cat $O/gemv_pmc.txt $O/mamba_pmc.txt | grep -v amdgpu
