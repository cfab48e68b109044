#!/bin/bash
# Push-relaxation A/B (verdict r03 item 1): the push variant's parity tests, then C4 and C5
# with the pull rounds (default) and the push rounds, interleaved, on one box.
set -o pipefail
export TMPDIR=/tmp
TAG=${1:?tag}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py -x -v --timeout 120 --timeout-method thread -m gpu -k "push" > $O/push_tests.log 2>&1
rc=$?; tail -3 $O/push_tests.log; [ $rc -ne 0 ] && { echo "push tests failed rc=$rc"; grep -E "FAILED|Error|assert" $O/push_tests.log | head -20; exit 1; }
for cfg in C4 C5; do
  for v in 1 2; do
    SHADOWTOPO_TRACE_ROUNDS=1 timeout -k 10 400 python -u bench.py --config $cfg --steps 3 --warmup 1 --no-cpu-baseline --no-host-rate --csr-variant $v > $O/bench_${cfg}_v$v.json 2> $O/bench_${cfg}_v$v.err || { echo "bench $cfg v$v failed"; tail -20 $O/bench_${cfg}_v$v.err; exit 1; }
    python3 scripts/bench_summary.py $O/bench_${cfg}_v$v.json
    python3 -c "import json,sys; d=json.load(open('$O/bench_${cfg}_v$v.json')); print('  phases', d['engine']['push_phases_ms_per_step'], 'syncs', d['engine']['host_syncs_per_step'])"
  done
done
