#!/bin/bash
# A/B bench lines: gpu_ab.sh TAG "args1" "args2" ... (each a bench.py argument string); prints ms/step + kernel ms
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-ab}
shift
i=0
for a in "$@"; do
  i=$((i+1))
  timeout -k 10 300 python -u bench.py --no-cpu-baseline $a > gpurun_out/ab_${TAG}_$i.json 2> gpurun_out/ab_${TAG}_$i.err || { echo "bench '$a' failed"; tail -5 gpurun_out/ab_${TAG}_$i.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; e=d['engine']; print(sys.argv[2], '| ms/step %.2f' % d['ms_per_step'], '| %s %.3f ms x %.1f' % (r['kernel'], r['avg_launch_ms'], r['launches_per_step']), '| delta', r.get('delta_kernel',{}).get('avg_launch_ms'), '| rounds', e['rounds_per_step'])" gpurun_out/ab_${TAG}_$i.json "$a"
done
