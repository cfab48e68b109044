#!/bin/bash
# r03 session 12: the pruned sweep's per-row loose bound (max thr - min W over the wave tile)
# in front of the full row filter -- parity of rf (6 waves/SIMD) and rf5 (5), A/B against head
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03l
mkdir -p $O
for v in rf rf5; do
  SHADOWTOPO_EXP_LIB=_exp/lib/libshadowtopo_$v.so timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py tests/test_fullsize_gpu.py -x -q --timeout 200 --timeout-method thread -m gpu -k "dense or c2" > $O/tests_$v.log 2>&1
  rc=$?; echo "$v: $(tail -1 $O/tests_$v.log)"; [ $rc -ne 0 ] && { echo "tests $v failed"; exit 1; }
done
B="--steps 10 --warmup 2 --no-cpu-baseline --no-host-rate --no-north-star"
for v in head rf rf5 head rf rf5; do
  export SHADOWTOPO_EXP_LIB=_exp/lib/libshadowtopo_$v.so
  timeout -k 10 200 python -u bench.py $B > $O/c2_$v.json 2> $O/c2_$v.err || { echo "c2 $v failed"; tail $O/c2_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/c2_$v.json')); r=d['roofline']; e=d['engine']; print('$v C2', round(d['ms_per_step'],3), 'sweep_ms', round(r['avg_launch_ms'],3), 'delta', round(r['delta_kernel']['avg_launch_ms'],3), 'cold', round(e['cold_start_ms'],1), e.get('cold_start_parts_ms'))"
done
