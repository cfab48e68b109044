#!/bin/bash
# r03 session 2: GPU suite (whole-matrix C3/C4 parity, lock-free cache shim), smoke, and
# the experiment variants (pred-gather cost, tile-major dense mapping)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03b
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -x -v --timeout 300 --timeout-method thread -m gpu --durations=15 > $O/gpu_tests.log 2>&1
rc=$?
tail -25 $O/gpu_tests.log
[ $rc -ne 0 ] && { echo "gpu tests failed rc=$rc"; exit 1; }
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; cat $O/smoke.log; exit 1; }
cat $O/smoke.log
B="--steps 10 --warmup 2 --no-cpu-baseline --no-host-rate --no-north-star"
for v in product nogather tilemajor dponly; do
  if [ $v = product ]; then unset SHADOWTOPO_EXP_LIB; else export SHADOWTOPO_EXP_LIB=_exp/lib/libshadowtopo_$v.so; fi
  if [ $v != dponly ]; then
  timeout -k 10 200 python -u bench.py $B > $O/c2_$v.json 2> $O/c2_$v.err || { echo "c2 $v failed"; tail $O/c2_$v.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('$O/c2_$v.json')); r=d['roofline']; print('$v C2', round(d['ms_per_step'],3), 'sweep', round(r['avg_launch_ms'],3), 'delta', r.get('delta_kernel'))"
  fi
  if [ $v != tilemajor ]; then
    timeout -k 10 200 python -u bench.py --config C4 --steps 3 --warmup 1 --no-cpu-baseline --no-host-rate --no-north-star > $O/c4_$v.json 2> $O/c4_$v.err || { echo "c4 $v failed"; tail $O/c4_$v.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open('$O/c4_$v.json')); r=d['roofline']; print('$v C4', round(d['ms_per_step'],3), 'relax', round(r['avg_launch_ms'],3), d['engine']['rounds_per_step'])"
  fi
done
unset SHADOWTOPO_EXP_LIB
timeout -k 10 400 python -u bench.py --steps 10 --warmup 2 > $O/bench_default.json 2> $O/bench_default.err || { echo "default bench failed"; tail -20 $O/bench_default.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_default.json')); print('default', d['ms_per_step'], d['value']); n=d['north_star']; print('north', n.get('matrix_build_ms'), {k: v['per_gpu_ms'] for k, v in n.get('projection', {}).items()}); print('shim', d['shim_host_matrix'])"
