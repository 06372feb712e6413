#!/bin/bash
# round 6, c2 (B = 1) layer: parity of the new B = 1 kernels, then the c2 decode step on the product
# library at 4 / 8 / 16 attention splits and on the round-5 sequence (variant b1old), then a kernel trace
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_fullwidth.py tests/test_gpu_generate.py -x -v \
    --timeout 300 --timeout-method thread -k "qkv_rope or q_part or out_proj_merge or c1 or c2 or c_decode_step" \
    > $O/tests.log 2>&1 && tail -n 1 $O/tests.log &&
timeout -k 10 300 python -u tools/c2_step.py 2 4 8 > $O/c2_product.log 2>&1 && grep "^c2" $O/c2_product.log &&
ZK_LIB_PATH=zonos_amd/lib/variants/b1old/libzonos_hip.so timeout -k 10 300 python -u tools/c2_step.py 4 \
    > $O/c2_old.log 2>&1 && grep "^c2" $O/c2_old.log &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
    python3 tools/c2_step.py 8 > $O/prof.log 2>&1 &&
find $O/prof -type f ! -name "*stats.csv" -delete
