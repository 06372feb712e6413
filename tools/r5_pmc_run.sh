set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5_pmc
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_hybrid.py -m gpu -q --timeout 300 --timeout-method thread > $O/hyb.log 2>&1
rc=$?; tail -n 2 $O/hyb.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $O/f -o run --output-format csv -- python3 tools/gemm_pmc.py > $O/f.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $O/w -o run --output-format csv -- python3 tools/gemm_pmc.py > $O/w.log 2>&1 &&
python tools/gemm_pmc.py --summary $O/f $O/w --json $O/r5_gemm_pmc.json &&
cp $O/r5_gemm_pmc.json profiles/ &&
find $O -name "*.csv" -path "*_SIZE*" -delete; 
timeout -k 10 600 python -u bench.py > $O/bench_c3.json.log 2>&1 && grep '^{' $O/bench_c3.json.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], json.dumps(d.get('gemm_roofline')))"
