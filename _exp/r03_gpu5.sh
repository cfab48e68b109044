#!/bin/bash
# r03 session 5: GPU suite after the cleanup, C5 with the pool-budget fix, C4, default bench
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03e
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -x -v --timeout 300 --timeout-method thread -m gpu --durations=8 > $O/gpu_tests.log 2>&1
rc=$?; tail -12 $O/gpu_tests.log; [ $rc -ne 0 ] && { echo "gpu tests failed"; exit 1; }
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; cat $O/smoke.log; exit 1; }
cat $O/smoke.log
for cfg in C5 C4; do
  timeout -k 10 400 python -u bench.py --config $cfg --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_$cfg.json 2> $O/bench_$cfg.err || { echo "$cfg failed"; tail $O/bench_$cfg.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench_$cfg.json')); e=d['engine']; print('$cfg', d['ms_per_step'], e['relax_ms_per_step'], e['engine_wall_ms_per_step'], e['pool_allocs_in_timed_steps'], e['cold_start_ms'], e['host_buffers_ms'])"
done
timeout -k 10 400 python -u bench.py --steps 10 --warmup 2 > $O/bench_default.json 2> $O/bench_default.err || { echo "default bench failed"; tail -20 $O/bench_default.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_default.json')); print('default', d['ms_per_step'], d['value']); n=d['north_star']; print('north', n.get('matrix_build_ms'), {k: v['per_gpu_ms'] for k, v in n.get('projection', {}).items()}); print('shim', d['shim_host_matrix']['prepare_ms'])"
