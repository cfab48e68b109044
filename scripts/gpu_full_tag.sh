#!/bin/bash
# full GPU suite, smoke, then host-path / cold-start benches for C3, C4, C2
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-x}
timeout -k 10 600 python -u -m pytest tests -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/gputests_$TAG.log 2>&1
rc=$?; tail -3 gpurun_out/gputests_$TAG.log
[ $rc -ne 0 ] && { echo "gpu tests failed rc=$rc"; grep -E "FAILED|Error|assert" gpurun_out/gputests_$TAG.log | head -20; exit 1; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/smoke_$TAG.log; exit 1; }
tail -1 gpurun_out/smoke_$TAG.log
for c in C3 C4 C2; do
  timeout -k 10 300 python -u bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/b_${TAG}_$c.json 2> gpurun_out/b_${TAG}_$c.err || { echo "bench $c failed"; tail -5 gpurun_out/b_${TAG}_$c.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/b_${TAG}_$c.json')); e=d['engine']; print('$c', round(d['ms_per_step'],2), 'host', e['host_buffers_ms'], 'pageable', e['host_buffers_pageable_ms'], 'cold', e['cold_start_ms'])"
  grep -E "engine \(graph" gpurun_out/b_${TAG}_$c.err
done
