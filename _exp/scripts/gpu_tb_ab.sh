#!/bin/bash
# Dense sweep batches per wave (OPT_DENSE_BATCHES_PER_WAVE 1 / 2): dense parity tests, then
# C2 interleaved on one box
set -o pipefail
export TMPDIR=/tmp
TAG=${1:?tag}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_engine_gpu.py tests/test_fullsize_gpu.py -x -q --timeout 200 --timeout-method thread -m gpu -k "dense or c2" > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" $O/tests.log | head -20; exit 1; }
for rep in 1 2; do
  for tb in 1 2; do
    timeout -k 10 300 python -u bench.py --steps 20 --warmup 2 --no-cpu-baseline --no-north-star --no-shim --no-host-rate --dense-tb $tb > $O/c2_tb${tb}_$rep.json 2> $O/c2_tb${tb}_$rep.err || { tail $O/c2_tb${tb}_$rep.err; exit 1; }
    echo -n "tb $tb rep $rep: "; python3 -c "import json; d=json.load(open('$O/c2_tb${tb}_$rep.json')); r=d['roofline']; print(round(d['ms_per_step'],4), 'sweep', round(r['avg_launch_ms'],4))"
  done
done
