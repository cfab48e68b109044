#!/bin/bash
# CSR source-order A/B: CSR GPU tests, then the C3 and C4 benches
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-csr}
timeout -k 10 400 python -u -m pytest tests/test_csr_gpu.py -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/gputests_$TAG.log 2>&1
rc=$?; tail -3 gpurun_out/gputests_$TAG.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" gpurun_out/gputests_$TAG.log | head -30; exit 1; }
for cfg in C3 C4; do
  timeout -k 10 400 python -u bench.py --config $cfg --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bench_${TAG}_$cfg.json 2> gpurun_out/bench_${TAG}_$cfg.err || { echo "bench $cfg failed"; tail -20 gpurun_out/bench_${TAG}_$cfg.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/bench_${TAG}_$cfg.json')); print('$cfg', d['ms_per_step'], d['engine']['rounds_per_step'])"
done
