#!/bin/bash
# per-wave key-slice trimming in the decode attention (product) vs whole blocks (variants/notrim)
set -e
export TMPDIR=/tmp
O=gpurun_out/trim
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_ops.py -k "attention or qkv or attn" > $O/t.log 2>&1
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_generate.py tests/test_gpu_step_small.py > $O/t2.log 2>&1
: > $O/ab.txt
for r in 1 2; do
  for v in product notrim; do
    lp=""; [ "$v" != product ] && lp=zonos_amd/lib/variants/$v/libzonos_hip.so
    echo "== $v" >> $O/ab.txt
    ZK_LIB_PATH=$lp ZK_MB_CTX=300,600,1000 timeout -k 10 200 python tools/microbench.py attn_small 2>&1 | grep "splits= 1" >> $O/ab.txt
    ZK_LIB_PATH=$lp timeout -k 10 200 python tools/microbench.py attn 2>&1 | grep "fused" >> $O/ab.txt
  done
done
for r in 1 2; do
  for v in product notrim; do
    lp=""; [ "$v" != product ] && lp=zonos_amd/lib/variants/$v/libzonos_hip.so
    ZK_LIB_PATH=$lp timeout -k 10 300 python -u bench.py --batch 1 --lc 160 --prefix 0 --new-tokens 861 --steps 2 --no-dac --no-cpu-baseline > $O/b.log 2>&1
    python -c "import json; d=json.loads([x for x in open('$O/b.log') if x.startswith('{')][-1]); print('$v c2 decode ms', d['breakdown']['decode_ms_per_token_step'])" >> $O/ab.txt
    ZK_LIB_PATH=$lp timeout -k 10 300 python -u bench.py --steps 1 --warmup 1 --no-dac --no-cpu-baseline > $O/b.log 2>&1
    python -c "import json; d=json.loads([x for x in open('$O/b.log') if x.startswith('{')][-1]); print('$v c3 decode ms', d['breakdown']['decode_ms_per_token_step'], d['roofline']['us_per_launch'])" >> $O/ab.txt
  done
done
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $O/pmc_f -o run --output-format csv -- python3 tools/attn_pmc.py > /dev/null 2>&1
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $O/pmc_w -o run --output-format csv -- python3 tools/attn_pmc.py > /dev/null 2>&1
python tools/pmc_summary.py $O/pmc_f $O/pmc_w > $O/pmc.txt 2>&1 || true
cat $O/ab.txt $O/pmc.txt
