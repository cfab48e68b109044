#!/bin/bash
# r03 session 36: pruned sweep visiting chunks outward on both sides of the tile (SHADOWTOPO_SWEEP_SPIRAL)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03ze
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_engine_gpu.py tests/test_fullsize_gpu.py -x -q --timeout 300 --timeout-method thread -m gpu -k "dense or c2" > $O/tests.log 2>&1
rc=$?; echo "tests: $(tail -1 $O/tests.log)"; [ $rc -ne 0 ] && { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
SHADOWTOPO_SWEEP_SPIRAL=1 timeout -k 10 400 python -u -m pytest tests/test_engine_gpu.py tests/test_fullsize_gpu.py -x -q --timeout 300 --timeout-method thread -m gpu -k "dense or c2" > $O/tests_spiral.log 2>&1
rc=$?; echo "tests spiral: $(tail -1 $O/tests_spiral.log)"; [ $rc -ne 0 ] && { echo "tests failed"; tail -30 $O/tests_spiral.log; exit 1; }
for run in "C2 1" "C2 0" "C2 1" "C2 0" "C2 1"; do
  set -- $run
  SHADOWTOPO_SWEEP_SPIRAL=$2 timeout -k 10 300 python -u bench.py --config $1 --steps 10 --warmup 2 --no-cpu-baseline --no-host-rate --no-north-star --no-shim > $O/$1_$2.json 2> $O/$1_$2.err || { echo "$run failed"; tail $O/$1_$2.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/$1_$2.json')); r=d['roofline']; print('$1 spiral=$2', round(d['ms_per_step'],3), 'sweep', round(r['avg_launch_ms'],3), 'delta', round(r['delta_kernel']['avg_launch_ms'],3))"
done
