#!/bin/bash
# full GPU suite, then sparse benches: "CFG:extra args" specs
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-sp}
shift
timeout -k 10 600 python -u -m pytest tests -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/gputests_$TAG.log 2>&1
rc=$?; tail -2 gpurun_out/gputests_$TAG.log
[ $rc -ne 0 ] && { echo "gpu tests failed rc=$rc"; grep -E "FAILED|Error|assert" gpurun_out/gputests_$TAG.log | head -20; exit 1; }
i=0
for spec in "$@"; do
  cfg=${spec%%:*}; a=${spec#*:}
  timeout -k 10 400 python -u bench.py --config $cfg --steps 2 --warmup 1 --no-cpu-baseline --no-host-rate $a > gpurun_out/b_${TAG}_$i.json 2> gpurun_out/b_${TAG}_$i.err || { echo "bench $spec failed"; tail -5 gpurun_out/b_${TAG}_$i.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/b_${TAG}_$i.json')); e=d['engine']; r=d['roofline']
print('$spec', round(d['ms_per_step'],2), 'rounds', e['rounds_per_step'], 'relax', round(e['relax_ms_per_step'],1), 'frac', round(r['frac'],4), 'batches', r['batches_per_launch'])"
  i=$((i+1))
done
