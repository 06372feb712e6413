# kernel-trace timelines of short c3 and c2 runs (per-kernel in-step durations and the gaps between
# consecutive kernels): tools/trace_gaps.py summarises them
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5_trace
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/c3 -o run -- python3 bench.py --steps 1 --warmup 0 --new-tokens 64 --no-dac --no-cpu-baseline > $O/c3.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/c2 -o run -- python3 bench.py --steps 1 --warmup 0 --batch 1 --lc 160 --prefix 0 --new-tokens 64 --no-dac --no-cpu-baseline > $O/c2.log 2>&1 &&
python3 tools/trace_gaps.py $O/c3 > $O/c3_gaps.txt && python3 tools/trace_gaps.py $O/c2 > $O/c2_gaps.txt && cat $O/c3_gaps.txt $O/c2_gaps.txt &&
find $O -name "*kernel_trace.csv" -size +20M -delete
