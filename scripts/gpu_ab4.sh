#!/bin/bash
# tests for the dense / CSR kernels, then one bench line per config (C2..C5) with round traces
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-ab}
timeout -k 10 500 python -u -m pytest tests/test_engine_gpu.py tests/test_csr_gpu.py tests/test_fullsize_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t_$TAG.log 2>&1
rc=$?; tail -2 gpurun_out/t_$TAG.log; [ $rc -ne 0 ] && exit $rc
for c in C2 C3 C4 C5; do
  st=10; [ $c = C5 ] && st=2
  SHADOWTOPO_TRACE_ROUNDS=1 timeout -k 10 300 python -u bench.py --config $c --steps $st --warmup 1 --no-cpu-baseline --no-host-rate --no-north-star > gpurun_out/b_${TAG}_$c.json 2> gpurun_out/b_${TAG}_$c.err || { echo "bench $c failed"; tail -5 gpurun_out/b_${TAG}_$c.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/b_${TAG}_$c.json'));r=d['roofline'];print('$c', round(d['ms_per_step'],3), r['kernel'], round(r['avg_launch_ms'],3), r.get('delta_kernel') or r.get('worklist_kernel'))"
done
