#!/bin/bash
# gpu tests + headline bench + extra bench invocations given as quoted arg strings
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-q}
shift
timeout -k 10 600 python -u -m pytest tests -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/gputests_$TAG.log 2>&1
rc=$?; tail -3 gpurun_out/gputests_$TAG.log
[ $rc -ne 0 ] && { echo "gpu tests failed rc=$rc"; grep -E "FAILED|Error|assert" gpurun_out/gputests_$TAG.log | head -20; exit 1; }
i=0
for a in "$@"; do
  i=$((i+1))
  timeout -k 10 400 python -u bench.py $a > gpurun_out/bench_${TAG}_$i.json 2> gpurun_out/bench_${TAG}_$i.err || { echo "bench '$a' failed"; tail -20 gpurun_out/bench_${TAG}_$i.err; exit 1; }
  echo "== $a"; cat gpurun_out/bench_${TAG}_$i.json
done
