#!/bin/bash
# CSR masked rounds: parity tests, then C3/C4 (and optionally C5) benches per variant
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-cm}
shift
timeout -k 10 400 python -u -m pytest tests/test_csr_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/csrtests_$TAG.log 2>&1
rc=$?; tail -3 gpurun_out/csrtests_$TAG.log
[ $rc -ne 0 ] && { echo "csr tests failed rc=$rc"; grep -E "FAILED|Error|assert" gpurun_out/csrtests_$TAG.log | head -20; exit 1; }
for spec in "$@"; do
  cfg=${spec%%:*}; v=${spec#*:}
  timeout -k 10 400 python -u bench.py --config $cfg --steps 2 --warmup 1 --no-cpu-baseline --no-host-rate --csr-variant $v > gpurun_out/b_${TAG}_${cfg}_$v.json 2> gpurun_out/b_${TAG}_${cfg}_$v.err || { echo "bench $cfg v$v failed"; tail -5 gpurun_out/b_${TAG}_${cfg}_$v.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/b_${TAG}_${cfg}_$v.json')); r=d['roofline']; e=d['engine']
print('$cfg v$v', round(d['ms_per_step'],2), 'rounds', e['rounds_per_step'], 'relax', round(e['relax_ms_per_step'],2), 'frac', r['frac'], 'avg', round(r['avg_launch_ms'],3))"
done
