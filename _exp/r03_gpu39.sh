#!/bin/bash
# r03 session 39: round-end check of the final tree -- GPU suite, smoke, default bench
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03zh
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -x -q --timeout 300 --timeout-method thread -m gpu > $O/gpu_tests.log 2>&1
rc=$?; tail -2 $O/gpu_tests.log; [ $rc -ne 0 ] && { echo "gpu tests failed"; exit 1; }
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; cat $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python -u bench.py --steps 10 --warmup 2 > $O/bench_default.json 2> $O/bench_default.err || { echo "default bench failed"; tail -20 $O/bench_default.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_default.json')); e=d['engine']; r=d['roofline']; print('default', d['ms_per_step'], d['value'], r['frac'], r['avg_launch_ms'], e['cold_start_ms']); n=d['north_star']; print('north', n.get('matrix_build_ms'))"
