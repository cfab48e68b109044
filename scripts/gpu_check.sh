#!/bin/bash
# full GPU test suite (incl. full-size parity) + headline bench: gpu_check.sh TAG [extra bench args]
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-chk}
shift
timeout -k 10 900 python -u -m pytest tests -x -v --timeout 300 --timeout-method thread -m gpu > gpurun_out/gputests_$TAG.log 2>&1
rc=$?; grep -E "passed|failed" gpurun_out/gputests_$TAG.log | tail -3
grep -E "PASSED|FAILED" gpurun_out/gputests_$TAG.log | grep -i "fullsize" 
[ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" gpurun_out/gputests_$TAG.log | head -20; exit 1; }
timeout -k 10 400 python -u bench.py "$@" > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { echo "bench failed"; tail -20 gpurun_out/bench_$TAG.err; exit 1; }
cat gpurun_out/bench_$TAG.json
