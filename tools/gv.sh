set -e
for v in wpacked nomfma noaload noboth; do
echo "== $v"; ZK_LIB_PATH=zonos_amd/lib/variants/$v/libzonos_hip.so timeout -k 10 120 python tools/microbench.py gemm 2>&1 | grep gemm
done
