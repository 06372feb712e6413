set -e
for v in att_noearly att_nokvw att_nopro; do
echo "== $v"; ZK_LIB_PATH=zonos_amd/lib/variants/$v/libzonos_hip.so timeout -k 10 120 python tools/microbench.py attn 2>&1 | grep "fused\|splits=1"
done
