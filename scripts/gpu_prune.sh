#!/bin/bash
# dense-sweep A/B: engine GPU tests, then the C2 bench
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-prune}
timeout -k 10 400 python -u -m pytest tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/gputests_$TAG.log 2>&1
rc=$?; tail -5 gpurun_out/gputests_$TAG.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" gpurun_out/gputests_$TAG.log | head -30; exit 1; }
timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { echo "bench failed"; tail -20 gpurun_out/bench_$TAG.err; exit 1; }
cat gpurun_out/bench_$TAG.json
