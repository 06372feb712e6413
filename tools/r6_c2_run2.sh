#!/bin/bash
# round 6 c2: attention parity, c2 step A/B over attention splits, stamps of the attention and GEMVs
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_fullwidth.py tests/test_gpu_generate.py -x -v \
    --timeout 300 --timeout-method thread -k "qkv_rope or q_part or out_proj_merge or c1 or c2 or c_decode_step" \
    > $O/tests.log 2>&1 && tail -n 1 $O/tests.log &&
timeout -k 10 300 python -u tools/c2_step.py 2 4 8 > $O/c2_product.log 2>&1 && grep "^c2" $O/c2_product.log &&
ZK_LIB_PATH=zonos_amd/lib/variants/attprof/libzonos_hip.so timeout -k 10 300 python tools/attn_b1_stamps.py \
    > $O/attn_stamps.txt 2>&1 && cat $O/attn_stamps.txt &&
ZK_LIB_PATH=zonos_amd/lib/variants/gfprof/libzonos_hip.so timeout -k 10 300 python tools/gemv_b1_stamps.py \
    > $O/gemv_stamps.txt 2>&1 && cat $O/gemv_stamps.txt
