#!/bin/bash
# One parametrised A/B / evidence driver for GPU boxes (replaces the round-1/2 one-off scripts).
#
#   tools/gpu_ab.sh OUT STEP [STEP ...]
#
# OUT is a directory under gpurun_out/. Each STEP runs under its own time limit, steps are
# chained (the first failure ends the run):
#   tests[:PYTEST_K]      pytest -m gpu (optionally -k PYTEST_K)
#   bench:NAME[:ARGS]     bench.py ARGS (comma-separated) -> OUT/bench_NAME.json.log
#   micro:MODE            tools/microbench.py MODE on the product library and every
#                         zonos_amd/lib/variants/<v> (built on the CPU with
#                         zonos_amd.build.build_variant), twice, interleaved
#   benchv:NAME[:ARGS]    bench.py ARGS on the product library and every variant, twice,
#                         interleaved -> OUT/benchv_NAME.log (value + decode ms per step)
#   testsv:PYTEST_K       pytest -m gpu -k PYTEST_K on every variant (parity must hold for any tuning)
#   prof:NAME[:ARGS]      rocprofv3 --kernel-trace --stats of bench.py ARGS -> OUT/prof_NAME/*stats.csv
#   pmcstd:ROUND          HBM bytes per launch of the decode attention (c3 shape, tools/attn_pmc.py) and
#                         the hybrid SSM step (c5 shape, microbench mamba): FETCH_SIZE / WRITE_SIZE in
#                         separate passes -> OUT/ROUND_{attn_fused,mamba_step}_pmc.{json,txt}
#   pmc:NAME:COUNTERS[:ARGS]  one rocprofv3 --pmc pass (COUNTERS comma-separated, within one
#                         block's limits) of bench.py ARGS -> OUT/pmc_NAME/
set -e
export TMPDIR=/tmp
OUT=gpurun_out/$1
shift
mkdir -p "$OUT"
for step in "$@"; do
  kind=${step%%:*}; rest=${step#*:}; [ "$rest" = "$step" ] && rest=""
  case "$kind" in
    tests)
      k=(); [ -n "$rest" ] && k=(-k "$rest")
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "${k[@]}" \
          > "$OUT/tests.log" 2>&1
      tail -n 1 "$OUT/tests.log" ;;
    bench)
      name=${rest%%:*}; a=${rest#*:}; [ "$a" = "$rest" ] && a=""
      timeout -k 10 600 python -u bench.py ${a//,/ } > "$OUT/bench_$name.json.log" 2>&1
      grep '^{' "$OUT/bench_$name.json.log" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$name', d['value'], d['unit'], d.get('breakdown'))" ;;
    micro)
      for i in 1 2; do
        echo "== product"; timeout -k 10 180 python tools/microbench.py $rest
        for v in $(ls zonos_amd/lib/variants 2>/dev/null); do
          echo "== $v"; ZK_LIB_PATH=zonos_amd/lib/variants/$v/libzonos_hip.so timeout -k 10 180 python tools/microbench.py $rest
        done
      done > "$OUT/micro_$rest.log" 2>&1
      grep -v amdgpu "$OUT/micro_$rest.log" ;;
    benchv)
      name=${rest%%:*}; a=${rest#*:}; [ "$a" = "$rest" ] && a=""
      for i in 1 2; do
        for v in product $(ls zonos_amd/lib/variants 2>/dev/null); do
          lp=""; [ "$v" != product ] && lp=zonos_amd/lib/variants/$v/libzonos_hip.so
          ZK_LIB_PATH=$lp timeout -k 10 400 python -u bench.py ${a//,/ } --no-cpu-baseline > "$OUT/benchv_tmp.log" 2>&1
          grep '^{' "$OUT/benchv_tmp.log" | python -c "import json,sys; d=json.loads(sys.stdin.read()); b=d['breakdown']; print('$v', d['value'], b.get('decode_ms_per_token_step'), b.get('dac_s_per_step'))"
        done
      done > "$OUT/benchv_$name.log" 2>&1
      rm -f "$OUT/benchv_tmp.log"
      cat "$OUT/benchv_$name.log" ;;
    testsv)
      for v in $(ls zonos_amd/lib/variants 2>/dev/null); do
        ZK_LIB_PATH=zonos_amd/lib/variants/$v/libzonos_hip.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q \
            --timeout 300 --timeout-method thread -k "$rest" > "$OUT/tests_$v.log" 2>&1
        echo "$v: $(tail -n 1 "$OUT/tests_$v.log")"
      done ;;
    pmcstd)
      for c in FETCH_SIZE WRITE_SIZE; do
        timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $c -d "$OUT/attn_$c" -o run --output-format csv -- \
            python3 tools/attn_pmc.py > "$OUT/attn_$c.log" 2>&1
        timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $c -d "$OUT/mamba_$c" -o run --output-format csv -- \
            python3 tools/microbench.py mamba > "$OUT/mamba_$c.log" 2>&1
      done
      python tools/pmc_summary.py "$OUT/attn_FETCH_SIZE" "$OUT/attn_WRITE_SIZE" --match "k_attn_decode<true" --R 128 \
          --ctx 1705 --alg 454033408 --json "$OUT/${rest}_attn_fused_pmc.json" > "$OUT/${rest}_attn_fused_pmc.txt"
      python tools/pmc_summary.py "$OUT/mamba_FETCH_SIZE" "$OUT/mamba_WRITE_SIZE" --match "k_mamba_step" --R 128 \
          --ctx 0 --alg 283803648 --json "$OUT/${rest}_mamba_step_pmc.json" > "$OUT/${rest}_mamba_step_pmc.txt"
      find "$OUT" -name "*.csv" -path "*_SIZE*" -delete
      cat "$OUT/${rest}_attn_fused_pmc.json" "$OUT/${rest}_mamba_step_pmc.json" ;;
    prof)
      name=${rest%%:*}; a=${rest#*:}; [ "$a" = "$rest" ] && a=""
      timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$name" -o run -- \
          python3 bench.py ${a//,/ } > "$OUT/prof_$name.log" 2>&1
      find "$OUT/prof_$name" -type f ! -name "*stats.csv" -delete ;;
    pmc)
      name=${rest%%:*}; r2=${rest#*:}; ctr=${r2%%:*}; a=${r2#*:}; [ "$a" = "$r2" ] && a=""
      timeout -s KILL 300 rocprofv3 --pmc ${ctr//,/ } --output-format csv -d "$OUT/pmc_$name" -o run -- \
          python3 bench.py ${a//,/ } > "$OUT/pmc_$name.log" 2>&1 ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
du -sh "$OUT"
