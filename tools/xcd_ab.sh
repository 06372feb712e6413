#!/bin/bash
# XCD-aware split-major tile order in k_gemm_ws (product) vs linear order (variants/noxcd)
set -e
export TMPDIR=/tmp
O=gpurun_out/xcd
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_ops.py -k "gemm" > $O/t.log 2>&1
: > $O/ab.txt
for r in 1 2; do
  for v in product noxcd; do
    lp=""; [ "$v" != product ] && lp=zonos_amd/lib/variants/$v/libzonos_hip.so
    echo "== $v" >> $O/ab.txt
    ZK_LIB_PATH=$lp timeout -k 10 200 python tools/microbench.py gemm 2>&1 | grep "^gemm" >> $O/ab.txt
  done
done
for r in 1 2; do
  for v in product noxcd; do
    lp=""; [ "$v" != product ] && lp=zonos_amd/lib/variants/$v/libzonos_hip.so
    ZK_LIB_PATH=$lp timeout -k 10 300 python -u bench.py --steps 1 --warmup 1 --no-dac --no-cpu-baseline > $O/b.log 2>&1
    python -c "import json; d=json.loads([x for x in open('$O/b.log') if x.startswith('{')][-1]); print('$v c3 decode ms', d['breakdown']['decode_ms_per_token_step'])" >> $O/ab.txt
  done
done
for v in product noxcd; do
  lp=""; [ "$v" != product ] && lp=zonos_amd/lib/variants/$v/libzonos_hip.so
  ZK_LIB_PATH=$lp timeout -s KILL 90 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $O/pf_$v -o run --output-format csv -- python3 tools/gemm_pmc.py > /dev/null 2>&1
  ZK_LIB_PATH=$lp timeout -s KILL 90 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $O/pw_$v -o run --output-format csv -- python3 tools/gemm_pmc.py > /dev/null 2>&1
  echo "== pmc $v" >> $O/ab.txt
  python tools/pmc_summary.py $O/pf_$v $O/pw_$v --match k_gemm_ws >> $O/ab.txt 2>&1 || true
done
cat $O/ab.txt
