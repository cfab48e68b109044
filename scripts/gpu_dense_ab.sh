#!/bin/bash
# dense parity tests, then the C2 bench (kernel times)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-d}
timeout -k 10 400 python -u -m pytest tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread -k "dense or geometric or prune" > gpurun_out/dtests_$TAG.log 2>&1
rc=$?; tail -2 gpurun_out/dtests_$TAG.log
[ $rc -ne 0 ] && { echo "dense tests failed rc=$rc"; grep -E "FAILED|Error|assert" gpurun_out/dtests_$TAG.log | head -20; exit 1; }
for i in 1 2; do
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-host-rate > gpurun_out/b_${TAG}_$i.json 2> gpurun_out/b_${TAG}_$i.err || { echo "bench failed"; tail -5 gpurun_out/b_${TAG}_$i.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/b_${TAG}_$i.json')); r=d['roofline']
print('C2', round(d['ms_per_step'],3), 'full', round(r['avg_launch_ms'],3), 'delta', round(r['delta_kernel']['avg_launch_ms'],3), 'x', r['delta_kernel']['launches_per_step'])"
done
