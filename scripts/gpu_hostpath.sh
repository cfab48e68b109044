#!/bin/bash
# engine + shim GPU tests, then the host-buffer (drop-in boundary) timings for C2/C3/C4
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-pin}
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py tests/test_topology_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_$TAG.log 2>&1
rc=$?; tail -3 gpurun_out/t_$TAG.log
[ $rc -ne 0 ] && { echo "tests failed rc=$rc"; grep -E "FAILED|Error|assert" gpurun_out/t_$TAG.log | head -20; exit 1; }
for c in C3 C4 C2; do
  timeout -k 10 300 python -u bench.py --config $c --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/b_${TAG}_$c.json 2> gpurun_out/b_${TAG}_$c.err || { echo "bench $c failed"; tail -5 gpurun_out/b_${TAG}_$c.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/b_${TAG}_$c.json')); e=d['engine']; print('$c', round(d['ms_per_step'],2), 'host', e['host_buffers_ms'], 'pageable', e['host_buffers_pageable_ms'], 'cold', e['cold_start_ms'])"
done
