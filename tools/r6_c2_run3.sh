#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 300 python -u tools/microbench.py gemv_warm > $O/gemv_warm.log 2>&1 && grep gemv_warm $O/gemv_warm.log &&
timeout -k 10 300 python -u tools/c2_step.py 4 > $O/c2_product.log 2>&1 && grep "^c2" $O/c2_product.log &&
ZK_LIB_PATH=zonos_amd/lib/variants/attprof/libzonos_hip.so timeout -k 10 300 python tools/attn_b1_stamps.py \
    > $O/attn_stamps.txt 2>&1 && cat $O/attn_stamps.txt
