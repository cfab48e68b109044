#!/bin/bash
# r03 session 16: the device build in the uploaded edge buffers -- GPU suite, smoke, default
# bench cold start (twice)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03p
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -x -q --timeout 300 --timeout-method thread -m gpu > $O/gpu_tests.log 2>&1
rc=$?; tail -2 $O/gpu_tests.log; [ $rc -ne 0 ] && { echo "gpu tests failed"; exit 1; }
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; cat $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
for k in 1 2; do
timeout -k 10 400 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-north-star > $O/bench_default$k.json 2> $O/bench_default$k.err || { echo "default bench failed"; tail -20 $O/bench_default$k.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_default$k.json')); e=d['engine']; print('default', d['ms_per_step'], d['value'], e['cold_start_ms'], e.get('cold_start_parts_ms'))"
done
