#!/bin/bash
# full GPU suite, then C5 (1M-vertex Chung-Lu, 50k sources) per CSR variant
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-c5}
shift
timeout -k 10 600 python -u -m pytest tests -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/gputests_$TAG.log 2>&1
rc=$?; tail -2 gpurun_out/gputests_$TAG.log
[ $rc -ne 0 ] && { echo "gpu tests failed rc=$rc"; grep -E "FAILED|Error|assert" gpurun_out/gputests_$TAG.log | head -20; exit 1; }
for v in "$@"; do
  timeout -k 10 400 python -u bench.py --config C5 --steps 1 --warmup 1 --no-cpu-baseline --no-host-rate --csr-variant $v > gpurun_out/b_${TAG}_C5_$v.json 2> gpurun_out/b_${TAG}_C5_$v.err || { echo "C5 v$v failed"; tail -5 gpurun_out/b_${TAG}_C5_$v.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/b_${TAG}_C5_$v.json')); e=d['engine']; r=d['roofline']
print('C5 v$v', round(d['ms_per_step'],1), 'rounds', e['rounds_per_step'], 'relax', round(e['relax_ms_per_step'],1), 'compose', round(e['compose_ms_per_step'],1), 'frac', r['frac'], 'cold', round(e['cold_start_ms']))"
done
