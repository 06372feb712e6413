#!/bin/bash
# B=1 attention: in-launch split combine with sc1 hand-off (product) vs release/acquire fences (variant)
set -e
export TMPDIR=/tmp
O=gpurun_out/sc1
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_ops.py -k "attention" > $O/t.log 2>&1
echo "== sc1 (product)" > $O/ab.txt
ZK_MB_CTX=300,600,1000 timeout -k 10 200 python tools/microbench.py attn_small 2>&1 | grep "splits" >> $O/ab.txt
echo "== fences" >> $O/ab.txt
ZK_LIB_PATH=zonos_amd/lib/variants/fence/libzonos_hip.so ZK_MB_CTX=300,600,1000 timeout -k 10 200 python tools/microbench.py attn_small 2>&1 | grep "splits" >> $O/ab.txt
cat $O/ab.txt
