#!/bin/bash
# r03 session 9: the 16-byte tree record {R, H, P} (one line per predecessor gather) --
# GPU suite on the product build, then A/B against v2 (separate H / R / P arrays) on C4, C3, C5
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03i
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -x -q --timeout 300 --timeout-method thread -m gpu --durations=5 > $O/gpu_tests.log 2>&1
rc=$?; tail -9 $O/gpu_tests.log; [ $rc -ne 0 ] && { echo "gpu tests failed"; exit 1; }
for run in "C4 v2" "C4 aos" "C4 v2" "C4 aos" "C3 v2" "C3 aos" "C5 v2" "C5 aos"; do
  set -- $run
  export SHADOWTOPO_EXP_LIB=_exp/lib/libshadowtopo_$2.so
  timeout -k 10 300 python -u bench.py --config $1 --steps 3 --warmup 1 --no-cpu-baseline --no-host-rate > $O/$1_$2.json 2> $O/$1_$2.err || { echo "$1 $2 failed"; tail $O/$1_$2.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/$1_$2.json')); e=d['engine']; r=d['roofline']; print('$1 $2', round(d['ms_per_step'],2), 'relax', round(e['relax_ms_per_step'],2), 'launch', round(r['avg_launch_ms'],3))"
done
