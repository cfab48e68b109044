#!/bin/bash
# r03 session 4: wave-independent dense sweep -- parity first, then A/B on C2; XCD-paired
# mapping; C5 again with the pool-allocation counters
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03d
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py -x -v --timeout 120 --timeout-method thread -m gpu -k "dense_wave or dense_prune or dense_seed" > $O/tests.log 2>&1
rc=$?; tail -12 $O/tests.log; [ $rc -ne 0 ] && { echo "tests failed"; exit 1; }
B="--steps 10 --warmup 2 --no-cpu-baseline --no-host-rate --no-north-star"
for sw in 0 1 0 1; do
  timeout -k 10 200 python -u bench.py $B --dense-sweep $sw > $O/c2_sweep$sw.json 2> $O/c2_sweep$sw.err || { echo "c2 sweep $sw failed"; tail $O/c2_sweep$sw.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/c2_sweep$sw.json')); r=d['roofline']; print('sweep=$sw C2', round(d['ms_per_step'],3), 'sweep_ms', round(r['avg_launch_ms'],3), 'delta', round(r['delta_kernel']['avg_launch_ms'],3))"
done
SHADOWTOPO_EXP_LIB=_exp/lib/libshadowtopo_xcdpair.so timeout -k 10 200 python -u bench.py $B > $O/c2_xcdpair.json 2> $O/c2_xcdpair.err || { echo "xcdpair failed"; tail $O/c2_xcdpair.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/c2_xcdpair.json')); r=d['roofline']; print('xcdpair C2', round(d['ms_per_step'],3), 'sweep_ms', round(r['avg_launch_ms'],3))"
timeout -k 10 400 python -u bench.py --config C5 --steps 3 --warmup 1 --no-cpu-baseline --no-host-rate > $O/bench_C5.json 2> $O/bench_C5.err || { echo "C5 failed"; tail $O/bench_C5.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_C5.json')); e=d['engine']; print('C5', d['ms_per_step'], e['relax_ms_per_step'], e['engine_wall_ms_per_step'], e['pool_allocs_in_timed_steps'], e['pool_alloc_ms_per_step'], e['cold_start_ms'])"
