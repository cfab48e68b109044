#!/bin/bash
# One config's measurement on the GPU box: kernel-trace stats + three separate PMC passes
# (FETCH_SIZE, WRITE_SIZE, SQ) over the SAME bench command, summarised into
# profiles/roofline_counters.json (key CFG@SCALE@1), then the bench line that reads them.
# usage: scripts/gpu_roofline.sh TAG CFG SCALE KERNEL_RE ["extra bench args"] [DISPATCHES_PER_LAUNCH]
# (KERNEL_RE: a Python regex over rocprof kernel names, e.g. "k_relax_dense_f<8, 2, 1, true>" or "k_relax<|k_relax_wl<" (the sparse relax kernels are templates)
# DISPATCHES_PER_LAUNCH: C2's sweep is 4 (chunk loop + exact pass, per part of OPT_SWEEP_PARTS = 2)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=$1
CFG=${2:-C2}
SCALE=${3:-1.0}
KERNEL=${4:-k_relax_dense_f<8, 2, 1, true>}
EXTRA=${5:-}
PER=${6:-1}
B="bench.py --config $CFG --scale $SCALE --steps 3 --warmup 1 --no-cpu-baseline --no-host-rate --no-north-star --no-fresh $EXTRA"
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt -o run --output-format csv -- python3 $B > $O/kt.json 2> $O/kt.err || { echo "kernel-trace failed"; tail -20 $O/kt.err; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $O/pf -o pmc --output-format csv -- python3 $B > $O/pf.json 2> $O/pf.err || { echo "pmc fetch failed"; tail -20 $O/pf.err; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d $O/pw -o pmc --output-format csv -- python3 $B > $O/pw.json 2> $O/pw.err || { echo "pmc write failed"; tail -20 $O/pw.err; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE -d $O/ps -o pmc --output-format csv -- python3 $B > $O/ps.json 2> $O/ps.err || { echo "pmc sq failed"; tail -20 $O/ps.err; exit 1; }
python3 scripts/roofline_counters.py "$CFG@$SCALE@1" "$KERNEL" $O/kt.json $O/pf $O/pw $O/ps $PER || exit 1
cp $O/kt/run_kernel_stats.csv $O/kernel_stats.csv 2>/dev/null || find $O/kt -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats.csv \;
cp profiles/roofline_counters.json $O/roofline_counters.json
timeout -k 10 300 python3 -u bench.py --config $CFG --scale $SCALE --steps 3 --warmup 1 --no-cpu-baseline $EXTRA > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
