#!/bin/bash
# GPU evidence run: the -m gpu suite (test failures do not stop the run; a crash, abort or time
# limit does), then gpu_ab.sh steps. Usage: tools/gpu_suite.sh OUT [gpu_ab.sh STEP ...]
export TMPDIR=/tmp
OUT=gpurun_out/$1
shift
mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > "$OUT/tests.log" 2>&1
rc=$?
tail -n 3 "$OUT/tests.log"
grep -E "FAILED|ERROR" "$OUT/tests.log" | head -20
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest exit $rc: stopping"; exit $rc; fi
[ $# -gt 0 ] && exec bash tools/gpu_ab.sh "$(basename "$OUT")" "$@"
exit 0
