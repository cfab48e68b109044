#!/bin/bash
# r03 session 15: drop-in GPU tests (directed-graph cache as the reference), engine tests, and
# the default bench's cold start with the staging-ring upload
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03o
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_topology_gpu.py tests/test_engine_gpu.py -x -q --timeout 200 --timeout-method thread -m gpu > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -ne 0 ] && { echo "tests failed"; exit 1; }
for k in 1 2; do
timeout -k 10 400 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-north-star > $O/bench_default$k.json 2> $O/bench_default$k.err || { echo "default bench failed"; tail -20 $O/bench_default$k.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_default$k.json')); e=d['engine']; print('default', d['ms_per_step'], d['value'], e['cold_start_ms'], e.get('cold_start_parts_ms'))"
done
