#!/bin/bash
# dense-variant sweep: gpu_variants.sh TAG "v1 v2 ..." [extra bench args]
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-var}
VARS=${2:-"0 2 3 4 5 6 7"}
EXTRA=${3:-}
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread -m gpu -k "variant or delta" > gpurun_out/vartests_$TAG.log 2>&1
rc=$?; tail -3 gpurun_out/vartests_$TAG.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" gpurun_out/vartests_$TAG.log | head -20; exit 1; }
for v in $VARS; do
  timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --dense-variant $v $EXTRA > gpurun_out/var_${TAG}_$v.json 2> gpurun_out/var_${TAG}_$v.err || { echo "variant $v failed"; tail -5 gpurun_out/var_${TAG}_$v.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print('variant', sys.argv[2], 'ms/step %.2f' % d['ms_per_step'], 'full %.2f' % r['avg_launch_ms'], 'delta', r.get('delta_kernel',{}).get('avg_launch_ms'))" gpurun_out/var_${TAG}_$v.json $v
done
