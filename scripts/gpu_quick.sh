#!/bin/bash
# quick GPU iteration: a pytest selection (-k expression), then optionally the default bench line.
#   scripts/gpu_quick.sh TAG "pytest -k expr" [bench]
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:?tag}
mkdir -p $O
if [ -n "$2" ]; then
  timeout -k 10 900 python -u -m pytest tests -x -v --timeout 300 --timeout-method thread -m gpu -k "$2" > $O/tests.log 2>&1
  rc=$?; tail -3 $O/tests.log; [ $rc -ne 0 ] && { echo "tests failed rc=$rc"; grep -E "FAILED|Error|error" $O/tests.log | head -20; exit 1; }
fi
if [ "$3" = bench ]; then
  timeout -k 10 500 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/bench_default.json 2> $O/bench_default.err || { echo "default bench failed"; tail -20 $O/bench_default.err; exit 1; }
  python3 scripts/bench_summary.py $O/bench_default.json
fi
exit 0
