set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5_pf
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py -m gpu -q --timeout 300 --timeout-method thread -k "gemm or prefill or swiglu" > $O/ops.log 2>&1
rc=$?; tail -n 3 $O/ops.log; grep -E "FAILED|Error" $O/ops.log | head
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for i in 1 2; do
  echo "== product"; timeout -k 10 180 python tools/microbench.py prefill || exit 1
  echo "== pfepi0"; ZK_LIB_PATH=zonos_amd/lib/variants/pfepi0/libzonos_hip.so timeout -k 10 180 python tools/microbench.py prefill || exit 1
done > $O/micro.log 2>&1
grep -v amdgpu $O/micro.log
timeout -k 10 180 python tools/prefill_lib_probe.py > $O/lib.log 2>&1; cat $O/lib.log
