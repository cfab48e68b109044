#!/bin/bash
# r03 session 19: the split sweep's chunk loop in 8-wave blocks (one staged D32 chunk for 8
# waves, 8 waves / SIMD) -- parity with SHADOWTOPO_SWEEP_NW=8, A/B against 4-wave blocks
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03s
mkdir -p $O
export SHADOWTOPO_EXP_LIB=_exp/lib/libshadowtopo_nw.so
SHADOWTOPO_SWEEP_NW=8 timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py tests/test_fullsize_gpu.py -x -q --timeout 200 --timeout-method thread -m gpu -k "dense or c2" > $O/tests_nw8.log 2>&1
rc=$?; echo "nw8: $(tail -1 $O/tests_nw8.log)"; [ $rc -ne 0 ] && { echo "tests failed"; exit 1; }
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py tests/test_fullsize_gpu.py -x -q --timeout 200 --timeout-method thread -m gpu -k "dense or c2" > $O/tests_nw4.log 2>&1
rc=$?; echo "nw4: $(tail -1 $O/tests_nw4.log)"; [ $rc -ne 0 ] && { echo "tests failed"; exit 1; }
B="--steps 10 --warmup 2 --no-cpu-baseline --no-host-rate --no-north-star"
for nw in 4 8 4 8; do
  export SHADOWTOPO_SWEEP_NW=$nw
  timeout -k 10 200 python -u bench.py $B > $O/c2_$nw.json 2> $O/c2_$nw.err || { echo "c2 $nw failed"; tail $O/c2_$nw.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/c2_$nw.json')); r=d['roofline']; print('nw=$nw C2', round(d['ms_per_step'],3), 'sweep_ms', round(r['avg_launch_ms'],3), 'delta', round(r['delta_kernel']['avg_launch_ms'],3))"
done
