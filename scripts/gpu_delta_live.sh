#!/bin/bash
# dense tests (incl. live-chunk delta rounds), then C2 with live lists never / auto, traced
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread -k "dense or geometric or prune or pinned or exchange" > gpurun_out/dl_tests.log 2>&1
rc=$?; tail -2 gpurun_out/dl_tests.log
[ $rc -ne 0 ] && { echo "tests failed rc=$rc"; grep -E "FAILED|Error|assert" gpurun_out/dl_tests.log | head -20; exit 1; }
for m in 0 2 0 2; do
  SHADOWTOPO_DELTA_LIVE=$m SHADOWTOPO_TRACE_ROUNDS=1 timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-host-rate > gpurun_out/dl_$m.json 2> gpurun_out/dl_$m.err || { echo "bench $m failed"; tail -5 gpurun_out/dl_$m.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/dl_$m.json')); r=d['roofline']
print('live=$m', round(d['ms_per_step'],3), 'full', round(r['avg_launch_ms'],3), 'delta', round(r['delta_kernel']['avg_launch_ms'],3), 'x', r['delta_kernel']['launches_per_step'])"
done
grep "round" gpurun_out/dl_2.err | tail -6
