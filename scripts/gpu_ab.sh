#!/bin/bash
# quick GPU check: a pytest selection, then bench lines for "CFG:extra args" specs
# usage: scripts/gpu_ab.sh TAG "PYTEST_ARGS" "C4:--csr-variant 1" ...
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=$1; shift
PT=$1; shift
if [ -n "$PT" ]; then
  timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread $PT > gpurun_out/pt_$TAG.log 2>&1
  rc=$?
  tail -4 gpurun_out/pt_$TAG.log
  [ $rc -ne 0 ] && { echo "pytest failed rc=$rc"; grep -E "Error|error|assert|FAILED" gpurun_out/pt_$TAG.log | head -30; exit 1; }
fi
i=0
for spec in "$@"; do
  i=$((i+1))
  cfg=${spec%%:*}; extra=${spec#*:}
  timeout -k 10 600 python -u bench.py --config $cfg --steps 3 --warmup 1 --no-cpu-baseline $extra > gpurun_out/ab_${TAG}_$i.json 2> gpurun_out/ab_${TAG}_$i.err || { echo "bench $spec failed"; tail -20 gpurun_out/ab_${TAG}_$i.err; exit 1; }
  python3 - "$spec" gpurun_out/ab_${TAG}_$i.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
r = d["roofline"]; e = d["engine"]
print(f"{sys.argv[1]:40s} {d['ms_per_step']:9.2f} ms/step  {r['kernel']} {r['avg_launch_ms']:.3f} ms x {r['launches_per_step']:.0f}  rounds {e['rounds_per_step']:.0f}  host {e['host_buffers_ms']}  cold {e['cold_start_ms']:.0f}")
PY
done
