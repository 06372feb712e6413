#!/bin/bash
# round 6 evidence: DAC per-kernel MFMA busy + HBM bytes (separate --pmc passes), c2 and c5 kernel traces
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
timeout -s KILL 240 rocprofv3 --kernel-trace --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv \
    -d $O/dac_mfma -o run -- python3 tools/dac_pmc.py > $O/dac_mfma.log 2>&1 &&
timeout -s KILL 240 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $O/dac_f -o run -- \
    python3 tools/dac_pmc.py > $O/dac_f.log 2>&1 &&
timeout -s KILL 240 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d $O/dac_w -o run -- \
    python3 tools/dac_pmc.py > $O/dac_w.log 2>&1 &&
python tools/mfma_summary.py $O/dac_mfma > $O/r6_dac_mfma_util_pmc.txt &&
python tools/pmc_by_kernel.py $O/dac_f $O/dac_w > $O/r6_dac_bytes_pmc.txt &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c2 -o run -- \
    python3 tools/c2_step.py 4 > $O/prof_c2.log 2>&1 &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c5 -o run -- \
    python3 bench.py --model hybrid --steps 1 --warmup 1 --no-cpu-baseline --no-secondary > $O/prof_c5.log 2>&1 &&
find $O -name "*.csv" ! -name "*stats.csv" -size +2M -delete
cat $O/r6_dac_mfma_util_pmc.txt $O/r6_dac_bytes_pmc.txt
