set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/profab
for i in 1 2; do
  for v in product attdma0; do
    lp=""; [ "$v" != product ] && lp=zonos_amd/lib/variants/$v/libzonos_hip.so
    ZK_LIB_PATH=$lp timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/profab/${v}_$i -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/profab/${v}_$i.log 2>&1
    find gpurun_out/profab/${v}_$i -type f ! -name "*kernel_stats.csv" -delete
    grep -h "k_attn_decode<true" gpurun_out/profab/${v}_$i/*kernel_stats.csv | cut -d, -f1-4 | sed "s/^/$v $i /"
  done
done
