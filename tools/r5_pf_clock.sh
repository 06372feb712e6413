# effective clock of the prefill GEMM with and without its MFMAs: GRBM_GUI_ACTIVE / 8 / duration
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/pfclk
for v in product pfnomfma; do
  lp=""; [ "$v" != product ] && lp=zonos_amd/lib/variants/$v/libzonos_hip.so
  ZK_LIB_PATH=$lp timeout -s KILL 120 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pfclk/$v -o run -- python3 tools/microbench.py prefill > gpurun_out/pfclk/$v.log 2>&1
done
find gpurun_out/pfclk -name "*.csv" | head
