#!/bin/bash
# device-driven rounds with the heavy-round grid traversal: parity, then A/B against the
# host-driven rounds on C4 groups (20 / 40 / all 157 batches), C3 and C5
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04m
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_csr_gpu.py -x -q --timeout 120 --timeout-method thread -m gpu > $O/csr_tests.log 2>&1
rc=$?; tail -2 $O/csr_tests.log; [ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" $O/csr_tests.log | head -20; exit 1; }
run() {
  timeout -k 10 300 python -u bench.py --config $1 --steps 3 --warmup 1 --no-cpu-baseline --no-host-rate $2 > $O/$3.json 2> $O/$3.err || { tail $O/$3.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/$3.json')); e=d['engine']; print('$3', round(d['ms_per_step'],2), 'relax', round(e['relax_ms_per_step'],2), 'rounds', e['rounds_per_step'], 'syncs', e['host_syncs_per_step'])"
}
for b in 20 40; do for d in 0 2; do run C4 "--batches $b --device-rounds $d" c4_b${b}_d$d || exit 1; done; done
for d in 0 2; do run C4 "--device-rounds $d" c4_all_d$d || exit 1; done
for d in 1 2; do run C3 "--device-rounds $d" c3_d$d || exit 1; done
for d in 0 2; do run C5 "--device-rounds $d" c5_d$d || exit 1; done
