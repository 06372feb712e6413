#!/bin/bash
# full GPU tests (with the hybrid full-geometry tests), c3 bench, prefill GEMM vs hipBLASLt probe
set -e
export TMPDIR=/tmp
O=gpurun_out/s4f2
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 500 --timeout-method thread > $O/tests.log 2>&1
timeout -k 10 500 python -u bench.py > $O/bench_c3.log 2>&1
timeout -k 10 120 python tools/microbench.py prefill > $O/prefill.txt 2>&1
timeout -k 10 120 python tools/blaslt_probe.py >> $O/prefill.txt 2>&1
tail -n 1 $O/tests.log
cat $O/prefill.txt | grep -v amdgpu
