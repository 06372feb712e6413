#!/bin/bash
# round 6: benchmark mode without the no-op EOS-resample launch (product) vs with it (withdraw1): parity, then c2
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    -k "generate or torch_noise or fullwidth or full_ or capi or hybrid or multirank or shard" > $O/tests.log 2>&1 && tail -n 1 $O/tests.log &&
for i in 1 2 3; do
  for v in product withdraw1; do
    lp=""; [ "$v" != product ] && lp=zonos_amd/lib/variants/$v/libzonos_hip.so
    ZK_LIB_PATH=$lp ZK_C2_REPS=2 timeout -k 10 300 python -u tools/c2_step.py 4 > $O/c2_$v.log 2>&1 || exit 1
    grep "^c2" $O/c2_$v.log | sed "s/^/$v /"
  done
done
