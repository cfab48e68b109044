#!/bin/bash
# r03 session 34: per-kernel FETCH/WRITE and SQ counters of the C2 step (PH1 vs PH2 vs delta)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03zc
mkdir -p $O
B="$GRAFT_REPO_ROOT/bench.py --config C2 --steps 3 --warmup 1 --no-cpu-baseline --no-host-rate --no-north-star --no-shim"
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $GRAFT_REPO_ROOT/$O/pf -o pmc --output-format csv -- python3 $B > $GRAFT_REPO_ROOT/$O/pf.json 2> $GRAFT_REPO_ROOT/$O/pf.err || { echo "pmc fetch failed"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $GRAFT_REPO_ROOT/$O/pw -o pmc --output-format csv -- python3 $B > $GRAFT_REPO_ROOT/$O/pw.json 2> $GRAFT_REPO_ROOT/$O/pw.err || { echo "pmc write failed"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_SALU -d $GRAFT_REPO_ROOT/$O/ps -o pmc --output-format csv -- python3 $B > $GRAFT_REPO_ROOT/$O/ps.json 2> $GRAFT_REPO_ROOT/$O/ps.err || { echo "pmc sq failed"; tail -5 $GRAFT_REPO_ROOT/$O/ps.err; exit 1; }
echo done
