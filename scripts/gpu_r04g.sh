#!/bin/bash
# W16 dense sweep A/B (verdict r03 item 4): parity tests, then C2 with the f32 and the fp16
# chunk loop interleaved, kernel times from the bench's HIP events
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04g
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py -x -v --timeout 120 --timeout-method thread -m gpu -k "w16 or dense_prune" > $O/w16_tests.log 2>&1
rc=$?; tail -3 $O/w16_tests.log; [ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" $O/w16_tests.log | head -20; exit 1; }
for rep in 1 2; do
  for w in 0 1; do
    timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-host-rate --no-north-star --dense-w16 $w > $O/c2_w${w}_$rep.json 2> $O/c2_w${w}_$rep.err || { echo "bench w16=$w failed"; tail -20 $O/c2_w${w}_$rep.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/c2_w${w}_$rep.json')); r=d['roofline']; print('w16=$w rep $rep', round(d['ms_per_step'],3), 'sweep', round(r['avg_launch_ms'],3), 'delta', round(r['delta_kernel']['avg_launch_ms'],3))"
  done
done
