#!/bin/bash
# MFMA utilisation of the DAC convs, the prefill GEMMs and the decode GEMMs on one GPU box:
# one rocprofv3 --pmc pass (SQ_VALU_MFMA_BUSY_CYCLES + GRBM_GUI_ACTIVE, within the SQ / GRBM limits)
# per program, each under its own time limit, summarised by tools/mfma_summary.py.
#   gpurun -- 'bash tools/mfma_pmc.sh'   ->  gpurun_out/r4s3_mfma/{dac,pf,gemm}_mfma.txt
# (timings printed by the programs under counter collection are not kernel times: rocprofv3
# serialises the dispatches it counts; the utilisation is per kernel over its own active cycles)
set -e
export TMPDIR=/tmp
O=gpurun_out/r4s3_mfma
mkdir -p $O
P="rocprofv3 --kernel-trace --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -o run"
timeout -s KILL 240 $P -d $O/dac -- python3 tools/dac_pmc.py > $O/dac.log 2>&1
timeout -s KILL 240 $P -d $O/pf -- python3 tools/microbench.py prefill > $O/pf.log 2>&1
timeout -s KILL 240 $P -d $O/gemm -- python3 tools/microbench.py gemm > $O/gemm.log 2>&1
python tools/mfma_summary.py $O/dac --match k_conv_cl > $O/dac_mfma.txt
python tools/mfma_summary.py $O/pf --match k_gemm_pf > $O/pf_mfma.txt
python tools/mfma_summary.py $O/gemm --match k_gemm_ws > $O/gemm_mfma.txt
find $O -name "*.csv" -size +5M -delete
cat $O/dac_mfma.txt $O/pf_mfma.txt $O/gemm_mfma.txt
