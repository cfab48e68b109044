#!/bin/bash
# kernel trace + FETCH_SIZE / WRITE_SIZE passes over one bench command (no summary)
#   scripts/gpu_prof.sh TAG "bench args"
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:?tag}
mkdir -p $O
B="bench.py $2"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt -o run --output-format csv -- python3 $B > $O/kt.json 2> $O/kt.err || { echo "kernel-trace failed"; tail -20 $O/kt.err; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $O/pf -o pmc --output-format csv -- python3 $B > $O/pf.json 2> $O/pf.err || { echo "pmc fetch failed"; tail -20 $O/pf.err; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d $O/pw -o pmc --output-format csv -- python3 $B > $O/pw.json 2> $O/pw.err || { echo "pmc write failed"; tail -20 $O/pw.err; exit 1; }
find $O -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $O/kernel_stats.csv
exit 0
