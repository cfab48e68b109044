#!/bin/bash
# r03 session 29b: build scratch freed after the dense allocation, one atomic per wave in k_complete
# parity subset, then cold start and step times on C2..C5
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03z5
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_engine_gpu.py tests/test_topology_gpu.py -x -q --timeout 300 --timeout-method thread -m gpu > $O/tests.log 2>&1
rc=$?; echo "tests: $(tail -1 $O/tests.log)"; [ $rc -ne 0 ] && { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
export SHADOWTOPO_TRACE_BUILD=1
for c in C2 C5 C2; do
  timeout -k 10 300 python -u bench.py --config $c --steps 5 --warmup 1 --no-cpu-baseline --no-host-rate --no-north-star --no-shim > $O/$c.json 2> $O/$c.err || { echo "$c failed"; tail $O/$c.err; exit 1; }
  echo "== $c"; grep -E "^\[(upload|create|graph_build)\]" $O/$c.err | tr '\n' ';'; echo
  python3 -c "import json; d=json.load(open('$O/$c.json')); e=d['engine']; print(round(d['ms_per_step'],3), 'sweep', round(d['roofline']['avg_launch_ms'],3), e['cold_start_parts_ms'], round(e['cold_start_ms'],1))"
done
