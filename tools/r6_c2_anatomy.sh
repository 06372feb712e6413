#!/bin/bash
# round 6 c2 anatomy on the current tree: B = 1 GEMV stamps (variant gfprof) and a rocprofv3 kernel trace
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
ZK_LIB_PATH=zonos_amd/lib/variants/gfprof/libzonos_hip.so timeout -k 10 300 python -u tools/gemv_b1_stamps.py > $O/gemv_stamps.txt 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c2 -o run -- \
    python3 tools/c2_step.py 4 > $O/prof_c2.log 2>&1 &&
find $O -name "*.csv" ! -name "*stats.csv" -size +2M -delete
cat $O/gemv_stamps.txt
