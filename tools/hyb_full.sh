#!/bin/bash
set -e
export TMPDIR=/tmp
O=gpurun_out/hybfull
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 500 --timeout-method thread tests/test_gpu_hybrid.py -k "full or mamba_step_kernel" > $O/t.log 2>&1
tail -n 20 $O/t.log
