set -e
for sp in "" "o=4,fc2=4" "o=4,fc2=4,qkv=2" "o=2,fc2=2,qkv=2,heads=1"; do
  echo "== splits [$sp]"
  ZK_SPLITS="$sp" timeout -k 10 300 python bench.py --steps 1 --warmup 1 --no-dac --no-cpu-baseline 2>&1 | grep '^{' | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['value'], d.get('breakdown',{}))"
done
