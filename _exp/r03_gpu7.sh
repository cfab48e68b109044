#!/bin/bash
# r03 session 7: perm entries prefetched a chunk ahead in the dense sweep -- parity, A/B against
# the r03e sweep, and two timing-only ablations (no filter: the chunk skeleton; no loads)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03g
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_engine_gpu.py tests/test_fullsize_gpu.py -x -v --timeout 200 --timeout-method thread -m gpu -k "dense or c2" > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -ne 0 ] && { echo "tests failed"; exit 1; }
B="--steps 10 --warmup 2 --no-cpu-baseline --no-host-rate --no-north-star"
for v in base pp base pp nofilter noload; do
  export SHADOWTOPO_EXP_LIB=_exp/lib/libshadowtopo_$v.so
  timeout -k 10 200 python -u bench.py $B > $O/c2_$v.json 2> $O/c2_$v.err || { echo "c2 $v failed"; tail $O/c2_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/c2_$v.json')); r=d['roofline']; print('$v C2', round(d['ms_per_step'],3), 'sweep_ms', round(r['avg_launch_ms'],3), 'delta', round(r['delta_kernel']['avg_launch_ms'],3))"
done
SHADOWTOPO_EXP_LIB=_exp/lib/libshadowtopo_phase.so timeout -k 10 120 python -u _exp/r03_phase.py > $O/phase.json 2> $O/phase.err || { echo phase failed; tail $O/phase.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/phase.json')); print('phase', d['span_us'], d['loop_us']['mean'], d['exact_us']['mean'], d['loop_us_per_chunk'], d['chunks_visited']['mean'], d['logged_rows_wave0']['mean'])"
