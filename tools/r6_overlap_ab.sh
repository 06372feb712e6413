#!/bin/bash
# c3 bench with the DAC serial vs overlapped with the next step's generate (side stream), interleaved
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
for i in 1 2; do
  for ov in 0 1; do
    timeout -k 10 400 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-secondary --dac-overlap $ov \
        > $O/bench_ov$ov.log 2>&1 || exit 1
    grep '^{' $O/bench_ov$ov.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); b=d['breakdown']; print('overlap', $ov, d['value'], d['ms_per_step'], b['generate_s_per_step'], b['dac_s_per_step'], b['dac_exposed_s_per_step'])"
  done
done
