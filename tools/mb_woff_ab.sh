#!/bin/bash
# SSM state written to a second buffer (variants/woff, ping-pong access pattern) vs in place
set -e
for i in 1 2 3; do
  for v in product woff; do
    lp=""; [ "$v" != product ] && lp=zonos_amd/lib/variants/$v/libzonos_hip.so
    echo "$v $(ZK_LIB_PATH=$lp timeout -k 10 120 python tools/microbench.py mamba 2>&1 | grep mamba_step)"
  done
done
