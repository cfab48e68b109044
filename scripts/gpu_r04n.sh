#!/bin/bash
# device rounds after the occupancy-sized grid and the 1 Mi bound: parity, C3 A/B (0/1/2),
# C4 20-batch group (0/2), and the default bench line (north-star projections)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04n
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_csr_gpu.py -x -q --timeout 120 --timeout-method thread -m gpu > $O/csr_tests.log 2>&1
rc=$?; tail -2 $O/csr_tests.log; [ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" $O/csr_tests.log | head -20; exit 1; }
run() {
  timeout -k 10 300 python -u bench.py --config $1 --steps 5 --warmup 1 --no-cpu-baseline --no-host-rate $2 > $O/$3.json 2> $O/$3.err || { tail $O/$3.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/$3.json')); e=d['engine']; print('$3', round(d['ms_per_step'],3), 'relax', round(e['relax_ms_per_step'],3), 'rounds', e['rounds_per_step'], 'syncs', e['host_syncs_per_step'])"
}
for rep in 1 2; do for d in 0 1 2; do run C3 "--device-rounds $d" c3_d${d}_$rep || exit 1; done; done
for d in 0 2; do run C4 "--batches 20 --device-rounds $d" c4_b20_d$d || exit 1; done
timeout -k 10 500 python -u bench.py --steps 10 --warmup 2 > $O/bench_default.json 2> $O/bench_default.err || { tail $O/bench_default.err; exit 1; }
python3 scripts/bench_summary.py $O/bench_default.json
