set -e
echo "== base"; timeout -k 10 120 python tools/microbench.py attn 2>&1 | grep "fused\|splits=1"
echo "== kvpacked"; ZK_LIB_PATH=zonos_amd/lib/variants/kvpacked/libzonos_hip.so timeout -k 10 120 python tools/microbench.py attn 2>&1 | grep "fused\|splits=1"
