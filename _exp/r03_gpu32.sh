#!/bin/bash
# r03 session 32: kernel trace of the C2 step (per-launch split of the delta rounds)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03za
mkdir -p $O
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/kt -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --config C2 --steps 4 --warmup 1 --no-cpu-baseline --no-host-rate --no-north-star --no-shim > $GRAFT_REPO_ROOT/$O/kt.json 2> $GRAFT_REPO_ROOT/$O/kt.err || { echo "trace failed"; tail $GRAFT_REPO_ROOT/$O/kt.err; exit 1; }
echo done
