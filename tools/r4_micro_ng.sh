set -e
export TMPDIR=/tmp
OUT=gpurun_out/r4_ng
mkdir -p $OUT
V=zonos_amd/lib/variants/ng2/libzonos_hip.so
for i in 1 2; do
  echo "== product default"; timeout -k 10 120 env ZK_MB_GEMM_EXTRA=fc1s:16384:2048:0 ZK_SPLITS=fc1s=2 python tools/microbench.py gemm
  echo "== ng2 qkv8 o8 fc2_16 fc1s2"; ZK_LIB_PATH=$V timeout -k 10 120 env ZK_MB_GEMM_EXTRA=fc1s:16384:2048:0 ZK_SPLITS=qkv=8,o=8,fc2=16,fc1s=2 python tools/microbench.py gemm
  echo "== ng2 qkv4 o16 fc2_8 fc1s4"; ZK_LIB_PATH=$V timeout -k 10 120 env ZK_MB_GEMM_EXTRA=fc1s:16384:2048:0 ZK_SPLITS=qkv=4,o=16,fc2=8,fc1s=4 python tools/microbench.py gemm
done 2>&1 | grep -v amdgpu.ids > $OUT/micro.log
cat $OUT/micro.log
