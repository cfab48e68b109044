#!/bin/bash
# r03 session 38: round-end product build after the spiral order and neighbour window -- GPU suite, smoke, C2 roofline refresh, C3-C5, default bench
# (the sweep = 2 dispatches: chunk loop + exact pass), C4 / C5 / default bench lines
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03zg
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -x -q --timeout 300 --timeout-method thread -m gpu > $O/gpu_tests.log 2>&1
rc=$?; tail -2 $O/gpu_tests.log; [ $rc -ne 0 ] && { echo "gpu tests failed"; exit 1; }
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; cat $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
bash scripts/gpu_roofline.sh r03zg_c2 C2 1.0 "k_relax_dense_f<8, 2, 1, true, [12], 4>" "" 2 > $O/roofline_c2.log 2>&1 || { echo "roofline c2 failed"; tail $O/roofline_c2.log; exit 1; }
tail -c 600 $O/roofline_c2.log; echo
for cfg in C3 C4 C5; do
  timeout -k 10 400 python -u bench.py --config $cfg --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_$cfg.json 2> $O/bench_$cfg.err || { echo "$cfg failed"; tail $O/bench_$cfg.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench_$cfg.json')); e=d['engine']; print('$cfg', round(d['ms_per_step'],2), round(e['relax_ms_per_step'],2), round(e['cold_start_ms']), e['host_buffers_ms'])"
done
timeout -k 10 400 python -u bench.py --steps 10 --warmup 2 > $O/bench_default.json 2> $O/bench_default.err || { echo "default bench failed"; tail -20 $O/bench_default.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_default.json')); e=d['engine']; r=d['roofline']; print('default', d['ms_per_step'], d['value'], r['frac'], r.get('traffic'), e['cold_start_ms']); n=d['north_star']; print('north', n.get('matrix_build_ms'))"
