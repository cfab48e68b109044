#!/bin/bash
# r03 session 28: where the staging ring's setup and the dense tables' time go (C2 create)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03z3
mkdir -p $O
export SHADOWTOPO_TRACE_BUILD=1
for run in "3 1" "3 0" "3 1"; do
  set -- $run
  SHADOWTOPO_UPLOAD_FILLERS=$1 SHADOWTOPO_PRELOAD=$2 timeout -k 10 300 python -u bench.py --config C2 --steps 2 --warmup 1 --no-cpu-baseline --no-host-rate --no-north-star > $O/p$2.json 2> $O/p$2.err || { echo "$run failed"; tail $O/p$2.err; exit 1; }
  echo "== fillers=$1 preload=$2"; grep -E "^\[(upload|create|graph_build)\]" $O/p$2.err | tr '\n' ';'; echo
  python3 -c "import json; d=json.load(open('$O/p$2.json')); print(d['engine']['cold_start_parts_ms'], d['engine']['cold_start_ms'])"
done
