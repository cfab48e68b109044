#!/bin/bash
# r03 session 25: where create()'s build phase goes (SHADOWTOPO_TRACE_BUILD phase stamps), C2 and C4
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03y
mkdir -p $O
export SHADOWTOPO_TRACE_BUILD=1
for c in C2 C4 C2; do
  timeout -k 10 300 python -u bench.py --config $c --steps 2 --warmup 1 --no-cpu-baseline --no-host-rate --no-north-star > $O/$c.json 2> $O/$c.err || { echo "$c failed"; tail $O/$c.err; exit 1; }
  echo "== $c"; grep -E "^\[(create|graph_build)\]" $O/$c.err
  python3 -c "import json; d=json.load(open('$O/$c.json')); print(d.get('cold_start_parts_ms'))"
done
