set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5_resid
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -m gpu -q --timeout 120 --timeout-method thread -k "resid" > $O/t.log 2>&1
rc=$?; tail -n 3 $O/t.log; grep -E "^E |Error" $O/t.log | head -20
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 180 python tools/microbench.py resid 2>&1 | grep -v amdgpu
timeout -k 10 180 python tools/microbench.py resid 2>&1 | grep -v amdgpu
