#!/bin/bash
# r03 session 37: a neighbour window after the tile's chunk in the sweep's chunk-skip evaluation (SHADOWTOPO_SWEEP_WIN1)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03zf
mkdir -p $O
SHADOWTOPO_SWEEP_WIN1=8 timeout -k 10 400 python -u -m pytest tests/test_engine_gpu.py tests/test_fullsize_gpu.py -x -q --timeout 300 --timeout-method thread -m gpu -k "dense or c2" > $O/tests.log 2>&1
rc=$?; echo "tests win1=8: $(tail -1 $O/tests.log)"; [ $rc -ne 0 ] && { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
for run in "C2 0" "C2 8" "C2 16" "C2 4" "C2 0" "C2 8" "C2 16"; do
  set -- $run
  SHADOWTOPO_SWEEP_WIN1=$2 timeout -k 10 300 python -u bench.py --config $1 --steps 10 --warmup 2 --no-cpu-baseline --no-host-rate --no-north-star --no-shim > $O/$1_$2.json 2> $O/$1_$2.err || { echo "$run failed"; tail $O/$1_$2.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/$1_$2.json')); r=d['roofline']; print('$1 win1=$2', round(d['ms_per_step'],3), 'sweep', round(r['avg_launch_ms'],3), 'delta', round(r['delta_kernel']['avg_launch_ms'],3))"
done
