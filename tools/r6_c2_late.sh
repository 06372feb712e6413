#!/bin/bash
# round 6 c2: B = 1 GEMV step words loaded first and tested only before the stores (ZK_GF_LATE=1, product) vs tested after the prefetch (nolate): parity, then c2, interleaved

set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_fullwidth.py tests/test_gpu_generate.py -x -v \
    --timeout 300 --timeout-method thread -k "qkv_rope or q_part or out_proj_merge or c1 or c2 or c_decode_step or gemv" \
    > $O/tests.log 2>&1 && tail -n 1 $O/tests.log &&
for i in 1 2 3; do
  for v in product nolate; do
    lp=""; [ "$v" != product ] && lp=zonos_amd/lib/variants/$v/libzonos_hip.so
    ZK_LIB_PATH=$lp ZK_C2_REPS=2 timeout -k 10 300 python -u tools/c2_step.py 4 > $O/c2_$v.log 2>&1 || exit 1
    grep "^c2" $O/c2_$v.log | sed "s/^/$v /"
  done
done
