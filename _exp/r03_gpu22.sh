#!/bin/bash
# r03 session 22: the dense epilogue's seed winners from permuted WI / WR rows (no WI / H / R gathers) -- parity, A/B
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03v
mkdir -p $O
SHADOWTOPO_EXP_LIB=_exp/lib/libshadowtopo_ep.so timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py tests/test_fullsize_gpu.py -x -q --timeout 200 --timeout-method thread -m gpu -k "dense or c2" > $O/tests_wp.log 2>&1
rc=$?; echo "ep: $(tail -1 $O/tests_wp.log)"; [ $rc -ne 0 ] && { echo "tests failed"; exit 1; }
B="--steps 10 --warmup 2 --no-cpu-baseline --no-host-rate --no-north-star"
for run in "head 2" "ep 2" "head 2" "ep 2"; do
  set -- $run
  export SHADOWTOPO_EXP_LIB=_exp/lib/libshadowtopo_$1.so SHADOWTOPO_SWEEP_XR=$2
  timeout -k 10 200 python -u bench.py $B > $O/c2_$1_$2.json 2> $O/c2_$1_$2.err || { echo "c2 $1 failed"; tail $O/c2_$1_$2.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/c2_$1_$2.json')); r=d['roofline']; print('$1 xr=$2 C2', round(d['ms_per_step'],3), 'sweep_ms', round(r['avg_launch_ms'],3), 'delta', round(r['delta_kernel']['avg_launch_ms'],3))"
done
