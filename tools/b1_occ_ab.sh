#!/bin/bash
# B=1 LN GEMVs: 2-row LDS image (product), one tile per workgroup (ZK_GF_B1_LAY1=1), occupancy variants
set -e
export TMPDIR=/tmp
O=gpurun_out/b1occ
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_ops.py -k "gemv or merge" > $O/t.log 2>&1
ZK_GF_B1_LAY1=1 ZK_LIB_PATH=zonos_amd/lib/variants/occ4pf4/libzonos_hip.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_ops.py -k "gemv" >> $O/t.log 2>&1
tail -n 1 $O/t.log > $O/ab.txt
run() {  # name, lib, lay1
  lp=""; [ "$2" != product ] && lp=zonos_amd/lib/variants/$2/libzonos_hip.so
  echo "== $1" >> $O/ab.txt
  ZK_LIB_PATH=$lp ZK_GF_B1_LAY1=$3 ZK_MB_M=2 ZK_MB_SHAPES=fc1:16384:2048:1:1,heads:9234:2048:0:1,qkv:3072:2048:0:1 timeout -k 10 120 python tools/microbench.py gemv 2>&1 | grep "^gemv" | cut -c1-60 >> $O/ab.txt
  ZK_LIB_PATH=$lp ZK_GF_B1_LAY1=$3 timeout -k 10 300 python -u bench.py --batch 1 --lc 160 --prefix 0 --new-tokens 861 --steps 2 --no-dac --no-cpu-baseline > $O/b.log 2>&1
  python -c "import json; d=json.loads([x for x in open('$O/b.log') if x.startswith('{')][-1]); print('$1 c2 decode ms', d['breakdown']['decode_ms_per_token_step'])" >> $O/ab.txt
}
for r in 1 2; do
  run prod_lay2 product 0
  run prod_lay1 product 1
  run occ4pf4_lay1 occ4pf4 1
  run occ3pf6_lay2 occ3pf6 0
done
ZK_GF_XR2=0 timeout -k 10 300 python -u bench.py --batch 1 --lc 160 --prefix 0 --new-tokens 861 --steps 2 --no-dac --no-cpu-baseline > $O/b.log 2>&1
python -c "import json; d=json.loads([x for x in open('$O/b.log') if x.startswith('{')][-1]); print('xr16 (old image) c2 decode ms', d['breakdown']['decode_ms_per_token_step'])" >> $O/ab.txt
cat $O/ab.txt
