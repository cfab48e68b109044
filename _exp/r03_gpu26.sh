#!/bin/bash
# r03 session 26: create() phases with/without the code-object preload thread; kernel stats of create
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03z
mkdir -p $O
export SHADOWTOPO_TRACE_BUILD=1
for run in "C2 0" "C2 1" "C4 0" "C4 1" "C2 1" "C2 0"; do
  set -- $run
  SHADOWTOPO_PRELOAD=$2 timeout -k 10 300 python -u bench.py --config $1 --steps 2 --warmup 1 --no-cpu-baseline --no-host-rate --no-north-star > $O/$1_$2.json 2> $O/$1_$2.err || { echo "$1 failed"; tail $O/$1_$2.err; exit 1; }
  echo "== $1 preload=$2"; grep -E "^\[(create|graph_build)\]" $O/$1_$2.err | tr '\n' ';'; echo
  python3 -c "import json; d=json.load(open('$O/$1_$2.json')); print(d['engine'].get('cold_start_parts_ms') or d.get('cold_start_parts_ms') or [k for k in d])"
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o c2 -- python3 $GRAFT_REPO_ROOT/bench.py --config C2 --steps 1 --warmup 0 --no-cpu-baseline --no-host-rate --no-north-star > $GRAFT_REPO_ROOT/$O/prof.log 2>&1 || { echo prof failed; tail $GRAFT_REPO_ROOT/$O/prof.log; exit 1; }
f=$(find $GRAFT_REPO_ROOT/$O/prof -name "*kernel_stats.csv" | head -1); cut -d, -f1-5 $f | head -30
